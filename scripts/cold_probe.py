"""Cold-cache probe of the headline vmult (Re3900 r2 FP64 Newton): what the
1 GiB scratch WRITE between reps (bench.py companions, `frac_cold`) costs the
timed vmult beyond taking the operator's data out of the MALL.

A write flush leaves the MALL and the L2s full of dirty lines of the scratch
buffer; the timed vmult's own reads then evict them, so their write-back to
HBM runs inside its events.  A READ of the same buffer evicts the operator's
data just as well and leaves clean lines.  Variants, alternated round by
round (medians of the per-call event times, one synchronize per call as in
the cold companion):
  warm          no flush
  write         scratch.fill_(1)                 (bench.py's cold flush)
  read          scratch viewed as float32, summed (1 GiB read, no dirty lines)
  write+read    the write flush, then the read flush
Usage: python scripts/cold_probe.py [reps_per_round] [rounds]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))

import torch  # noqa: E402

import bench  # noqa: E402
import glsamd  # noqa: E402
import glsinputs as gi  # noqa: E402
import glsmesh as gm  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    d = gm.read_deck(os.path.join(gm.DECK_DIR, bench.DECK))
    mesh = d.mesh(d.n_refinements)
    vel, p, slip = d.boundary_descriptor()
    cmask = mesh.constraint_mask(vel, p, slip)
    params, weights = d.operator_parameters(2.5e-4)
    u_star = gi.linearization_point(mesh.n_nodes, mesh.dim, d.u_max)
    op = glsamd.NavierStokesOperator(mesh, cmask, "f64")
    op.set_parameters(**params)
    op.set_linearization_point(u_star)
    if params["order"] > 0:
        op.set_previous_solution(gi.history(u_star, params["order"]), weights)
    src = op._dev(gi.src_vector(mesh.n_dofs))
    dst = op.initialize_dof_vector()
    b = bench.survey_bytes(op)

    scratch = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    f32 = scratch.view(torch.float32)
    sink = torch.zeros((), dtype=torch.float32, device="cuda")

    def write():
        scratch.fill_(1)

    def read():
        torch.sum(f32, dim=0, out=sink)

    def write_read():
        write()
        read()

    variants = {"warm": None, "write": write, "read": read, "write+read": write_read}
    for _ in range(200):  # clock settle (bench.py --settle-ms)
        op.vmult(dst, src)
    torch.cuda.synchronize()
    times = {k: [] for k in variants}
    for r in range(rounds):
        for name, fl in variants.items():
            for _ in range(5):
                op.vmult(dst, src)
            t = []
            for _ in range(reps):
                if fl is not None:
                    fl()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                op.vmult(dst, src)
                e1.record()
                torch.cuda.synchronize()
                t.append(e0.elapsed_time(e1))
            times[name].append(float(np.median(t)))
            print(f"round {r} {name:11s} {times[name][-1] * 1e3:8.2f} us", flush=True)
    # does a READ allocate in the MALL (so that the read flush evicts)?  A
    # 128 MiB buffer summed right after a 1 GiB read flush (from HBM), then
    # again at once (from the MALL if reads allocate there)
    a = torch.ones(32 << 20, dtype=torch.float32, device="cuda")
    sa = torch.zeros((), dtype=torch.float32, device="cuda")
    cold_a, warm_a = [], []
    for _ in range(10):
        read()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        torch.sum(a, dim=0, out=sa)
        e[1].record()
        torch.sum(a, dim=0, out=sa)
        e[2].record()
        torch.cuda.synchronize()
        cold_a.append(e[0].elapsed_time(e[1]))
        warm_a.append(e[1].elapsed_time(e[2]))
    nb = a.numel() * 4
    ca, wa = float(np.median(cold_a)), float(np.median(warm_a))
    print(f"# MALL read allocation: 128 MiB sum after the 1 GiB read flush {ca * 1e3:.1f} us "
          f"({nb / ca / 1e9:.2f} TB/s), the same sum again {wa * 1e3:.1f} us "
          f"({nb / wa / 1e9:.2f} TB/s)")
    print(f"# Re3900 r2 FP64 Newton vmult, {mesh.n_dofs} DoFs, SURVEY 8d bytes {b:.0f}; "
          f"medians of {reps} synchronised calls per round, {rounds} rounds")
    print(f"{'variant':11s} {'us (rounds)':>40s} {'frac':>7s}")
    for name, v in times.items():
        m = float(np.median(v))
        print(f"{name:11s} {' '.join(f'{x * 1e3:7.2f}' for x in v):>40s} "
              f"{b / (m * 1e-3) / bench.HBM_PEAK:7.3f}")


if __name__ == "__main__":
    main()
