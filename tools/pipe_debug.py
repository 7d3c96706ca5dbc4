"""Debug driver for the multi-stream paths: one small batch per configuration, progress on stderr."""
import faulthandler
import os
import sys

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import of_dis_amd as od  # noqa: E402

w, h, n = 320, 240, 5
pairs = [od.synth_pair(w, h, 1, f, 1) for f in range(n)]
a = torch.from_numpy(np.stack([x[0] for x in pairs])).cuda()
b = torch.from_numpy(np.stack([x[1] for x in pairs])).cuda()
p = od.oppoint(2, w, 1, 1)
ctx = od.Context(0)
ref = ctx.run(a, b, p)
torch.cuda.synchronize()
ref = ref.cpu().numpy()
for cfg in sys.argv[1:]:
    chunk, graph, pipeline, streams = (int(x) for x in cfg.split(","))
    print("config chunk=%d graph=%d pipeline=%d streams=%d" % (chunk, graph, pipeline, streams), file=sys.stderr,
          flush=True)
    ctx.set_option("streams", streams)
    ctx.set_option("chunk", chunk)
    ctx.set_option("graph", graph)
    ctx.set_option("pipeline", pipeline)
    for rep in range(2):
        o = ctx.run(a, b, p)
        torch.cuda.synchronize()
        on = o.cpu().numpy()
        same = [bool(np.array_equal(on[f].view(np.uint32), ref[f].view(np.uint32))) for f in range(n)]
        diff = [float(np.abs(on[f] - ref[f]).max()) for f in range(n)]
        print("  rep %d same=%s maxdiff=%s" % (rep, same, diff), file=sys.stderr, flush=True)
ctx.close()
