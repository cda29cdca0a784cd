#!/usr/bin/env python3
"""Dev: time tools/sweep_ceiling.hip — the Jacobian sweep's exact traffic (B x 304 B read, B x 3968 B
written) moved by an ideal streaming kernel — the same way bench.jacobian_sweep times the sweep (back-to-back launches
between one HIP event pair behind a spin kernel), next to the sweep itself.  Prints one JSON line.

  python tools/sweep_ceiling.py [B=65536] [reps=20]        (build: python tools/sweep_ceiling.py --build, on the CPU)
"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tools", "_sweep_ceiling.so")


def build():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", SO,
                           os.path.join(ROOT, "tools", "sweep_ceiling.hip")])


def main():
    if "--build" in sys.argv:
        build()
        return
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    import torch
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
    L = ctypes.CDLL(SO)
    dev = torch.device("cuda", 0)
    inp = torch.randn(B * 304 // 8, dtype=torch.float64, device=dev)
    out = torch.empty(B * 3968 // 8, dtype=torch.float64, device=dev)
    blocks = ctypes.c_int(0)
    assert L.ceiling_resident(ctypes.byref(blocks)) == 0
    st = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(st.cuda_stream)

    def launch():
        rc = L.ceiling_launch(ctypes.c_void_p(inp.data_ptr()), ctypes.c_void_p(out.data_ptr()), ctypes.c_longlong(B),
                              blocks.value, sp)
        assert rc == 0, rc
    for _ in range(3):
        launch()
    torch.cuda.synchronize(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if hasattr(torch.cuda, "_sleep"):
        with torch.cuda.stream(st):
            torch.cuda._sleep(int(2e7))
    a.record(st)
    for _ in range(reps):
        launch()
    b.record(st)
    torch.cuda.synchronize(dev)
    ms = a.elapsed_time(b) / reps
    byts = B * (304 + 3968)
    rep = {"kernel": "stream_kernel (tools/sweep_ceiling.hip)", "batch": B, "grid": blocks.value, "ms": ms,
           "bytes": byts, "GBs": byts / (ms * 1e-3) / 1e9, "frac_of_8TBs": byts / (ms * 1e-3) / 8e12}
    # the fill's order (r6): the same bytes streamed front to back by the whole grid, 8 workgroups of 4 waves per CU
    fb = ctypes.c_int(0)
    assert L.fill_order_resident(ctypes.byref(fb)) == 0

    def launch_f():
        rc = L.fill_order_launch(ctypes.c_void_p(inp.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                 ctypes.c_longlong(B), fb.value, sp)
        assert rc == 0, rc
    for _ in range(3):
        launch_f()
    torch.cuda.synchronize(dev)
    if hasattr(torch.cuda, "_sleep"):
        with torch.cuda.stream(st):
            torch.cuda._sleep(int(2e7))
    a.record(st)
    for _ in range(reps):
        launch_f()
    b.record(st)
    torch.cuda.synchronize(dev)
    fms = a.elapsed_time(b) / reps
    rep.update({"fill_order_kernel_grid": fb.value, "fill_order_ms": fms, "fill_order_GBs": byts / (fms * 1e-3) / 1e9,
                "fill_order_frac_of_8TBs": byts / (fms * 1e-3) / 8e12})
    # and torch's own fill of the output buffer (the runtime's fill kernel), the same way
    for _ in range(2):
        out.fill_(1.0)
    torch.cuda.synchronize(dev)
    if hasattr(torch.cuda, "_sleep"):
        with torch.cuda.stream(st):
            torch.cuda._sleep(int(2e7))
    a.record(st)
    for _ in range(reps):
        out.fill_(1.0)
    b.record(st)
    torch.cuda.synchronize(dev)
    zms = a.elapsed_time(b) / reps
    rep.update({"torch_fill_out_ms": zms, "torch_fill_out_GBs": B * 3968 / (zms * 1e-3) / 1e9})
    import bench
    import alipmpc
    from alipmpc import scenes

    class A:
        sweep_batch = B
        seed = 0
    r = bench.jacobian_sweep(alipmpc, scenes, alipmpc.VARIANT_MODI, A, dev, reps=reps)
    rep["sweep_ms"] = r["kernel_ms"]
    rep["sweep_GBs"] = r["achieved"]
    rep["sweep_frac_of_ceiling"] = r["achieved"] / rep["GBs"]
    print(json.dumps(rep))


if __name__ == "__main__":
    main()
