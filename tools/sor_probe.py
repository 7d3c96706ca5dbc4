#!/usr/bin/env python3
"""Where a wavefront step of the exact-order SOR spends its time.

Loads the probe build of the library (tools/bin/libofdis_sorprobe.so: `make -C of_dis_amd/csrc probe`,
kernels compiled with -DOFDIS_SOR_PROBE), runs n 1080p op-point-2 pairs through its C-ABI on one stream,
and reads the per-step shader-clock records frame 0 of every k_tv_sor_lanes launch wrote:

    t0 after the previous step's barrier   t1 the step's LDS operands have arrived
    t2 its update written to LDS            t3 after the step's barrier

so a step = lds (t1 - t0: ring / coefficient-ring reads incl. the wait behind the barrier's release)
+ valu (t2 - t1: the update chain and the ring write) + barrier (t3 - t2: waiting for the slowest wave).
Reports medians per level and wave role, in cycles of the shader clock (s_memtime), and the probe's own
ns per step from HIP events.

    python tools/sor_probe.py [n_pairs ...] > gpurun_out/.../sor_probe.json      (GPU box)
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SLOTS, WAVES, STEPS = 64, 16, 1024


def main():
    import torch
    from of_dis_amd import _lib
    import of_dis_amd as od

    lib = C.CDLL(os.path.join(ROOT, "tools", "bin", "libofdis_sorprobe.so"))
    vp = C.c_void_p
    lib.ofdis_sor_probe_attach.argtypes = [vp]
    lib.ofdis_context_create.argtypes = [C.c_int, C.POINTER(vp)]
    lib.ofdis_context_destroy.argtypes = [vp]
    lib.ofdis_context_set_option.argtypes = [vp, C.c_char_p, C.c_int]
    lib.ofdis_run_batch_u8.argtypes = [vp, vp, vp, C.c_int, C.c_int, C.c_int, C.POINTER(_lib.Params), vp, vp]
    torch.cuda.set_device(0)
    W, H = 1920, 1080
    p = od.oppoint(2, W, od.MODE_OF, 1)
    p.verbosity = 0
    levels = list(range(p.sc_f, p.sc_l - 1, -1))
    # every k_tv_sor_lanes launch records a slot: all levels in order
    launches = [s for s in levels for _ in range(p.tv_innerit * (s + 1))]  # refine_variational.cpp:36
    out = {"what": __doc__.split("\n\n")[0], "clock": "s_memtime (shader clock)", "runs": []}
    ctx = vp()
    assert lib.ofdis_context_create(0, C.byref(ctx)) == 0
    for key, val in (("graph", 0), ("streams", 1)):
        lib.ofdis_context_set_option(ctx, key.encode(), val)
    ns = [int(x) for x in sys.argv[1:]] or [1, 32, 1024]
    for n in ns:
        a1, b1 = od.synth_pair(W, H, 1, 0, od.MODE_OF)
        a = torch.from_numpy(np.stack([a1] * n)).cuda()
        b = torch.from_numpy(np.stack([b1] * n)).cuda()
        flow = torch.empty((n, H, W, 2), dtype=torch.float32, device="cuda")
        rec = torch.zeros(4 + SLOTS * WAVES * STEPS * 4, dtype=torch.int32, device="cuda")
        run = lambda: lib.ofdis_run_batch_u8(ctx, a.data_ptr(), b.data_ptr(), n, W, H, C.byref(p),  # noqa: E731
                                             flow.data_ptr(), torch.cuda.current_stream().cuda_stream)
        assert lib.ofdis_sor_probe_attach(None) == 0
        for _ in range(3):
            assert run() == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert run() == 0  # unprobed, for the wall time of the call
        e1.record()
        torch.cuda.synchronize()
        call_ms = e0.elapsed_time(e1)
        assert lib.ofdis_sor_probe_attach(C.c_void_p(rec.data_ptr())) == 0
        assert run() == 0
        torch.cuda.synchronize()
        assert lib.ofdis_sor_probe_attach(None) == 0
        r = rec.cpu().numpy().view(np.uint32)
        nl = int(r[0])
        recs = r[4:].reshape(SLOTS, WAVES, STEPS, 4).astype(np.int64)
        per_level = {}
        for li in range(min(nl, SLOTS)):
            lv = launches[li] if li < len(launches) else -1
            w, h = (W >> lv, (H + 8) >> lv) if lv >= 0 else (0, 0)  # 1080 padded to 1088 (2^6)
            for wv in range(WAVES):
                R = recs[li, wv]
                live = R[:, 3] != 0
                if not live.any():
                    continue
                R = R[live]
                d = (R - R[:, :1]) % (1 << 32)
                S = p.tv_solverit
                role = f"{lv}:sweep{wv % S}"  # wave wid = g * S + s (sor_lanes_frame)
                for key in (lv, role):
                    if key not in per_level:
                        per_level[key] = {"size": f"{w}x{h}", "lds": [], "valu": [], "barrier": [], "step": [],
                                          "gap": [], "waves": set()}
                ent = per_level[role]
                ent["waves"].add(wv)
                d = (R - R[:, :1]) % (1 << 32)
                ent["lds"] += list(d[:, 1])
                ent["valu"] += list(d[:, 2] - d[:, 1])
                ent["barrier"] += list(d[:, 3] - d[:, 2])
                ent = per_level[lv]
                ent["waves"].add(wv)
                ent["lds"] += list(d[:, 1])
                ent["valu"] += list(d[:, 2] - d[:, 1])
                ent["barrier"] += list(d[:, 3] - d[:, 2])
                t3 = R[:, 3]
                ent["step"] += list(np.diff(t3) % (1 << 32))
                ent["gap"] += list((R[1:, 0] - R[:-1, 3]) % (1 << 32))
        summ = {}
        for lv, e in sorted(per_level.items(), key=lambda kv: str(kv[0]), reverse=True):
            summ[str(lv)] = {"size": e["size"], "waves": len(e["waves"]),
                             **{k: {"median": float(np.median(e[k])), "p90": float(np.percentile(e[k], 90))}
                                for k in ("step", "lds", "valu", "barrier", "gap") if e[k]}}
        out["runs"].append({"pairs": n, "call_ms": call_ms, "sor_launches_recorded": nl, "levels": summ})
        print(json.dumps(out["runs"][-1]), file=sys.stderr, flush=True)
    lib.ofdis_context_destroy(ctx)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
