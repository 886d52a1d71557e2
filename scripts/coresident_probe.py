"""Co-residency probe (measurement only, DESIGN.md §7 "frames in flight"):
while one C3 psrt_trace launch runs (ctx stream), launch small 64-thread
workgroups on another stream 3 ms later and report when they got a CU slot,
relative to the trace launch's enqueue (s_memrealtime, 10 ns ticks).

usage: python scripts/coresident_probe.py <probe.so>"""
import ctypes as C
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import petershirleyraytracer_amd as P  # noqa: E402


def main():
    lib = C.CDLL(sys.argv[1])
    lib.probe_launch.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_uint, C.c_int]
    scene, cam = P.scene_random_spheres(1), P.camera_look_at(aspect=1.5)
    ctx = P.Context(0)
    ctx.set_scene(scene, cam)
    prm = P.params(1200, 800, 100, 50, 0, 0, 1)
    acc = torch.zeros((800, 1200, 3), dtype=torch.float64, device="cuda")
    s2 = torch.cuda.Stream()
    base = torch.zeros(1, dtype=torch.int64, device="cuda")
    end = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.render_device(prm, acc.data_ptr(), 0, ctx.stream())
    ctx.sync_stats()
    out = []
    for nwg, spin, prio, delay in [(256, 0, 0, 0.003), (1024, 5000, 0, 0.003),
                                   (1024, 5000, 1, 0.003), (4096, 0, 0, 0.003),
                                   (1024, 5000, 0, None)]:
        st = torch.zeros(nwg, dtype=torch.int64, device="cuda")
        lib.probe_launch(C.c_void_p(s2.cuda_stream), C.c_void_p(base.data_ptr()), 1, 0, 0)
        torch.cuda.synchronize()
        if delay is not None:
            ctx.render_device(prm, acc.data_ptr(), 0, ctx.stream())
            lib.probe_launch(C.c_void_p(ctx.stream()), C.c_void_p(end.data_ptr()), 1, 0, 0)
            time.sleep(delay)
        lib.probe_launch(C.c_void_p(s2.cuda_stream), C.c_void_p(st.data_ptr()), nwg, spin, prio)
        torch.cuda.synchronize()
        if delay is not None:
            ctx.sync_stats()
        b = int(base.item())
        t = sorted((int(x) - b) / 100.0 for x in st.cpu().tolist())  # microseconds
        q = lambda f: round(t[min(len(t) - 1, int(f * len(t)))], 1)
        row = {"wgs": nwg, "spin_ticks": spin, "prio3": prio, "beside_trace": delay is not None,
               "start_us_p0_p10_p50_p90_p100": [q(0), q(0.1), q(0.5), q(0.9), t[-1]],
               "trace_end_us": round((int(end.item()) - b) / 100.0, 1) if delay else None}
        out.append(row)
        print(json.dumps(row), flush=True)
    # VGPR budget beside the trace: kernels holding N floats live
    lib.probe_vgpr_launch.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_uint, C.c_int]
    lib.probe_sgpr_launch.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_uint, C.c_int]
    for kind, n in [("v", 8), ("v", 26), ("s", 4), ("s", 12), ("s", 20), ("s", 28)]:
        st = torch.zeros(1024, dtype=torch.int64, device="cuda")
        lib.probe_launch(C.c_void_p(s2.cuda_stream), C.c_void_p(base.data_ptr()), 1, 0, 0)
        torch.cuda.synchronize()
        ctx.render_device(prm, acc.data_ptr(), 0, ctx.stream())
        lib.probe_launch(C.c_void_p(ctx.stream()), C.c_void_p(end.data_ptr()), 1, 0, 0)
        time.sleep(0.003)
        fn = lib.probe_vgpr_launch if kind == "v" else lib.probe_sgpr_launch
        fn(C.c_void_p(s2.cuda_stream), C.c_void_p(st.data_ptr()), 1024, 5000, n)
        torch.cuda.synchronize()
        ctx.sync_stats()
        b = int(base.item())
        t = sorted((int(x) - b) / 100.0 for x in st.cpu().tolist())
        print(json.dumps({"live": kind + "gpr", "n": n, "start_us_p0_p50_p100": [t[0], t[len(t) // 2], t[-1]],
                          "trace_end_us": round((int(end.item()) - b) / 100.0, 1)}), flush=True)
    # the lean reduce's loop on C3-sized synthetic records, alone and beside a trace
    lib.probe_reduce_launch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint, C.c_uint,
                                        C.c_void_p, C.c_void_p, C.c_int]
    S, npx = 100, 960000
    tt = torch.rand(npx * S, dtype=torch.float64, device="cuda")
    kk = torch.randint(0, 6, (npx * S,), dtype=torch.int16, device="cuda")
    nwg = (npx + 63) // 64
    stamps = torch.zeros(2 * nwg, dtype=torch.int64, device="cuda")
    sums = torch.zeros(npx, dtype=torch.float64, device="cuda")
    for beside, prio in [(False, 0), (False, 1), (True, 0), (True, 1)]:
        lib.probe_launch(C.c_void_p(s2.cuda_stream), C.c_void_p(base.data_ptr()), 1, 0, 0)
        torch.cuda.synchronize()
        if beside:
            ctx.render_device(prm, acc.data_ptr(), 0, ctx.stream())
            lib.probe_launch(C.c_void_p(ctx.stream()), C.c_void_p(end.data_ptr()), 1, 0, 0)
            time.sleep(0.003)
        lib.probe_reduce_launch(C.c_void_p(s2.cuda_stream), C.c_void_p(tt.data_ptr()),
                                C.c_void_p(kk.data_ptr()), S, npx, C.c_void_p(stamps.data_ptr()),
                                C.c_void_p(sums.data_ptr()), prio)
        torch.cuda.synchronize()
        if beside:
            ctx.sync_stats()
        b = int(base.item())
        sv = stamps.cpu().view(-1, 2).tolist()
        starts = sorted((s0 - b) / 100.0 for s0, _ in sv)
        ends = sorted((e - b) / 100.0 for _, e in sv)
        durs = sorted((e - s0) / 100.0 for s0, e in sv)
        q = lambda t, f: round(t[min(len(t) - 1, int(f * len(t)))], 1)
        row = {"reduce_loop": True, "beside_trace": beside, "prio3": prio,
               "first_start_us": q(starts, 0), "last_end_us": q(ends, 1),
               "wg_us_p10_p50_p90": [q(durs, 0.1), q(durs, 0.5), q(durs, 0.9)],
               "trace_end_us": round((int(end.item()) - b) / 100.0, 1) if beside else None}
        print(json.dumps(row), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
