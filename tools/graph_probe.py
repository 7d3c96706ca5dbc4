#!/usr/bin/env python3
"""Graph capture of the multi-lane issues (option graph=2), one configuration per child process so a crash
names its configuration.  Usage: python tools/graph_probe.py [streams,chunk,pipeline[,pipe_skip] ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import faulthandler, sys, numpy as np, torch
faulthandler.enable()
sys.path.insert(0, %r)
import of_dis_amd as od
streams, chunk, pipeline = %d, %d, %d
w, h, n = 320, 240, 5
pairs = [od.synth_pair(w, h, 1, f, 1) for f in range(n)]
a = torch.from_numpy(np.stack([x[0] for x in pairs])).cuda()
b = torch.from_numpy(np.stack([x[1] for x in pairs])).cuda()
p = od.oppoint(2, w, 1, 1)
ctx = od.Context(0)
ctx.set_option("streams", streams); ctx.set_option("chunk", chunk); ctx.set_option("pipeline", pipeline)
ctx.set_option("graph", 0)
ref = ctx.run(a, b, p); torch.cuda.synchronize(); ref = ref.cpu().numpy()
ctx.set_option("graph", 3 if pipeline else 2)
for rep in range(3):
    o = ctx.run(a, b, p); torch.cuda.synchronize()
    print("rep", rep, "same", np.array_equal(o.cpu().numpy().view(np.uint32), ref.view(np.uint32)), flush=True)
ctx.close()
'''
cfgs = sys.argv[1:] or ["3,2,0", "1,2,1", "2,3,0"]
rc_all = 0
for c in cfgs:
    s, ch, pl, *sk = (int(x) for x in c.split(","))
    env = dict(os.environ, OFDIS_TRACE="1", OFDIS_PIPE_SKIP=str(sk[0] if sk else 0))
    r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, s, ch, pl)], env=env, capture_output=True, text=True,
                       timeout=120)
    print(f"== streams {s} chunk {ch} pipeline {pl} skip {sk}: rc {r.returncode}")
    print(r.stdout[-1500:])
    print(r.stderr[-3000:])
    rc_all = rc_all or r.returncode
    if r.returncode not in (0, 1):
        break
sys.exit(0 if rc_all in (0, 1) else rc_all)
