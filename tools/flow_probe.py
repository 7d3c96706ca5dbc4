#!/usr/bin/env python3
"""Where the dataflow TV iteration (k_tv_flow, of_dis_amd/csrc/ofdis_tvflow.hip) spends its time.

Loads the probe build (tools/bin/libofdis_flowprobe.so: `make -C of_dis_amd/csrc fprobe`, the flow kernel compiled
with -DOFDIS_FLOW_PROBE; never loaded by the package, the tests or bench.py), runs n 1080p op-point-2 pairs on one
stream and reads what frame 0 of every k_tv_flow launch recorded per wave and loop iteration: shader clock at the
iteration's start (t0), when its wait held (t1), after it published (t2), and the polls it took.

Per level and role (SOR sweep s, M = rows + smoothness, Y = system): median iteration period (t2[i+1] - t2[i]),
wait (t1 - t0), work (t2 - t1), polls; and the launch span (first t0 .. last t2) in cycles.

    python tools/flow_probe.py [n_pairs ...] > gpurun_out/.../flow_probe.json      (GPU box)
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SLOTS, WAVES, ITERS = 64, 16, 256


def roles(h, S=3):
    G, NM, P = 1, 3, 12 - S
    r = {}
    for s in range(S):
        for g in range(G):
            r[s * G + g] = f"sor{s}_g{g}"
    r[S * G] = "L"
    for m in range(NM):
        r[S + 1 + m] = f"M{m}"
    for j in range(P):
        r[S + 1 + NM + j] = f"Y{j}"
    return r


def main():
    import torch
    from of_dis_amd import _lib
    import of_dis_amd as od

    lib = C.CDLL(os.path.join(ROOT, "tools", "bin", "libofdis_flowprobe.so"))
    vp = C.c_void_p
    lib.ofdis_flow_probe_attach.argtypes = [vp]
    lib.ofdis_context_create.argtypes = [C.c_int, C.POINTER(vp)]
    lib.ofdis_context_destroy.argtypes = [vp]
    lib.ofdis_context_set_option.argtypes = [vp, C.c_char_p, C.c_int]
    lib.ofdis_run_batch_u8.argtypes = [vp, vp, vp, C.c_int, C.c_int, C.c_int, C.POINTER(_lib.Params), vp, vp]
    torch.cuda.set_device(0)
    W, H = 1920, 1080
    p = od.oppoint(2, W, od.MODE_OF, 1)
    p.verbosity = 0
    levels = list(range(p.sc_f, p.sc_l - 1, -1))
    launches = [s for s in levels for _ in range(p.tv_innerit * (s + 1))]
    out = {"what": __doc__.split("\n\n")[0], "clock": "s_memtime (shader clock)", "runs": []}
    ctx = vp()
    assert lib.ofdis_context_create(0, C.byref(ctx)) == 0
    opts = [("graph", 0), ("streams", 1)] + [(kv.split("=")[0], int(kv.split("=")[1]))
                                             for kv in os.environ.get("FLOW_PROBE_OPTS", "").split(",") if kv]
    for key, val in opts:
        assert lib.ofdis_context_set_option(ctx, key.encode(), val) == 0, key
    ns = [int(x) for x in sys.argv[1:]] or [1, 32]
    for n in ns:
        a1, b1 = od.synth_pair(W, H, 1, 0, od.MODE_OF)
        a = torch.from_numpy(np.stack([a1] * n)).cuda()
        b = torch.from_numpy(np.stack([b1] * n)).cuda()
        flow = torch.empty((n, H, W, 2), dtype=torch.float32, device="cuda")
        rec = torch.zeros(4 + SLOTS * WAVES * ITERS * 4, dtype=torch.int32, device="cuda")
        run = lambda: lib.ofdis_run_batch_u8(ctx, a.data_ptr(), b.data_ptr(), n, W, H, C.byref(p),  # noqa: E731
                                             flow.data_ptr(), torch.cuda.current_stream().cuda_stream)
        assert lib.ofdis_flow_probe_attach(None) == 0
        for _ in range(3):
            assert run() == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert run() == 0
        e1.record()
        torch.cuda.synchronize()
        call_ms = e0.elapsed_time(e1)
        assert lib.ofdis_flow_probe_attach(C.c_void_p(rec.data_ptr())) == 0
        assert run() == 0
        torch.cuda.synchronize()
        assert lib.ofdis_flow_probe_attach(None) == 0
        r = rec.cpu().numpy().view(np.uint32)
        nl = int(r[0])
        recs = r[4:].reshape(SLOTS, WAVES, ITERS, 4).astype(np.int64)
        run_out = {"pairs": n, "call_ms_unprobed": round(call_ms, 4), "launches": nl, "levels": {}}
        for li in range(min(nl, len(launches))):
            s = launches[li]
            w, h = W >> s, -(-H // (1 << s))
            key = f"{w}x{h}"
            lv = run_out["levels"].setdefault(key, {"launch_span_cycles": [], "roles": {}})
            R = recs[li]
            t0s = R[:, :, 0][R[:, :, 2] > 0]
            t2s = R[:, :, 2][R[:, :, 2] > 0]
            if len(t2s):
                lv["launch_span_cycles"].append(int(t2s.max() - t0s.min()))
            for wv, name in roles(h).items():
                rr = R[wv]
                m = rr[:, 2] > 0
                if m.sum() < 4:
                    continue
                rr = rr[m]
                per = np.diff(rr[:, 2])
                st = lv["roles"].setdefault(name, {"period": [], "wait": [], "work": [], "polls": [], "iters": []})
                st["period"].append(float(np.median(per)))
                st["wait"].append(float(np.median(rr[:, 1] - rr[:, 0])))
                st["work"].append(float(np.median(rr[:, 2] - rr[:, 1])))
                st["polls"].append(float(np.mean(rr[:, 3])))
                st["iters"].append(int(m.sum()))
        for key, lv in run_out["levels"].items():
            lv["launch_span_cycles"] = int(np.median(lv["launch_span_cycles"]))
            for name, st in lv["roles"].items():
                for k in list(st):
                    st[k] = round(float(np.median(st[k])), 1)
        out["runs"].append(run_out)
    lib.ofdis_context_destroy(ctx)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
