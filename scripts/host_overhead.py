"""Host-side cost of one vmult call and the fixed cost of bench.py's timed
region (GPU box).  Prints one JSON object.

  call_us       CPU time of op.vmult() while the GPU is busy (queue not full)
  parts_us      its pieces: torch current-stream lookup, two data_ptr()s,
                the bare C-ABI call with prepared arguments
  region        perf_counter around K vmults (+ the two region events, as
                bench.py does) vs the events' own duration, median of reps:
                the difference is the launch latency + synchronize wake-up
"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import glsamd  # noqa: E402
import glsinputs as gi  # noqa: E402
import glsmesh as gm  # noqa: E402


def main():
    d = gm.read_deck(os.path.join(gm.DECK_DIR, "input_hoffmann_3D_Re3900.json"))
    mesh = d.mesh(d.n_refinements)
    vel, p, slip = d.boundary_descriptor()
    cm = mesh.constraint_mask(vel, p, slip)
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(mesh.n_nodes, mesh.dim, d.u_max)
    op = glsamd.NavierStokesOperator(mesh, cm, "f64")
    op.set_parameters(**params)
    op.set_linearization_point(u)
    if params["order"] > 0:
        op.set_previous_solution(gi.history(u, params["order"]), w)
    src = op._dev(gi.src_vector(mesh.n_dofs))
    dst = op.initialize_dof_vector()
    for _ in range(10):
        op.vmult(dst, src)
    torch.cuda.synchronize()

    def busy_cpu(fn, n=30):
        torch.cuda._sleep(200_000_000)  # keep the GPU busy: enqueues never block
        t = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            t.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        return float(np.median(t)) * 1e6

    lib = glsamd.lib()
    h = op.h
    pd, ps = C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr())
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = {"call_us": busy_cpu(lambda: op.vmult(dst, src)),
           "parts_us": {
               "current_stream": busy_cpu(lambda: torch.cuda.current_stream().cuda_stream, 200),
               "raw_stream": busy_cpu(lambda: torch._C._cuda_getCurrentRawStream(
                   torch.cuda.current_device()), 200),
               "glsamd_stream": busy_cpu(glsamd._stream, 200),
               "two_data_ptr": busy_cpu(lambda: (dst.data_ptr(), src.data_ptr()), 200),
               "c_abi_call": busy_cpu(lambda: lib.gls_op_vmult(h, pd, ps, sp)),
               "event_record": busy_cpu(lambda: torch.cuda.Event(enable_timing=True).record(),
                                        200)}}
    reg = {}
    for K in (20, 50):
        wall, ev = [], []
        for _ in range(15):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(K):
                op.vmult(dst, src)
            e1.record()
            torch.cuda.synchronize()
            wall.append((time.perf_counter() - t0) * 1e3)
            ev.append(e0.elapsed_time(e1))
        wm, em = float(np.median(wall)), float(np.median(ev))
        reg[f"K{K}"] = {"wall_ms": wm, "events_ms": em, "fixed_us": (wm - em) * 1e3,
                        "ms_per_step_wall": wm / K, "ms_per_step_events": em / K}
    out["region"] = reg
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
