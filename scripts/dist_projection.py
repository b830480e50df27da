#!/usr/bin/env python3
"""Per-rank projection of the partitioned multigrid at N = 1, 2, 4, 8 GPUs
(unmeasured on more than one GPU: this runs on ONE).

For each world size the Re3900 r0..r2 hierarchy is partitioned as the
multi-GPU bench partitions it (glsdist.coarse_bounds / build_partitions:
every level on the same coarse cells) and the LARGEST rank's local work is
timed with no exchange: a single-domain FP32 multigrid on that rank's cells
of every level (glsdist.LocalMesh, the rank-local child lattices), the same
smoother and 10 coarse relaxation sweeps as the bench's V-cycle companion;
its FP64 local vmult; and a GMRES(28) iteration on the rank's cells.  The
agglomerated variant (levels r0, r1 run redundantly and single-domain on
every rank) is timed as the rank's r2 work (a two-level local
hierarchy r1..r2 whose coarse solve is a copy) plus the global r0..r1
V-cycle.  Exchange phases per V-cycle are counted from the algorithm
(csrc/dist_mg.hip v_step): every partitioned level apply has an import and
an export phase, every level pair a compress and a ghost update; the
projection adds them at an exposed cost per phase EPS (the measured
in-process device-copy floor of profiles/r05/dist/threaded_vmult_overlap.txt,
and RCCL-like latencies), and the agglomerated cycle's all-reduce of the
level-r1 right-hand side (global r1 vector) at a ring-all-reduce cost.
Prints one JSON object per world size and a summary table.
    python scripts/dist_projection.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import glsamd  # noqa: E402
import glsdist  # noqa: E402
import glsinputs as gi  # noqa: E402
import glsmesh as gm  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 30
NS = 5          # smoothing steps per level (Multigrid default, the decks' 5)
COARSE = 10     # coarse relaxation sweeps (the bench's V-cycle companion)
EPS_US = (4.2, 10.0, 20.0)  # exposed cost per halo phase (floor: in-process copies)
XGMI_GBS = 50.0             # effective per-link all-reduce bandwidth assumed (GB/s)


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def local_levels(meshes, cmasks, parts, r, levels):
    lms = [glsdist.LocalMesh(meshes[l], parts[l][r]) for l in levels]
    lcm = [np.ascontiguousarray(np.asarray(cmasks[l])[parts[l][r].local_nodes]) for l in levels]
    child = glsdist.rank_child_lattices(meshes, parts, r)
    ch = [np.ascontiguousarray(np.asarray(child[l], dtype=np.uint32) & np.uint32(0x7FFFFFFF))
          for l in levels[1:]]
    return lms, lcm, ch


def multigrid(lms, lcm, ch, params, u_f, h_f, w, coarse):
    ops = []
    for m, c in zip(lms, lcm):
        op = glsamd.NavierStokesOperator(m, c, "f32")
        op.set_parameters(**params)
        ops.append(op)
    mg = glsamd.Multigrid(ops, ch, smoothing_n_iterations=NS, coarse_n_iterations=coarse)
    vecs = [ops[-1]._dev(u_f)]
    hists = [[ops[-1]._dev(h) for h in h_f]]
    for l in range(len(ops) - 1, 0, -1):
        v = ops[l - 1].initialize_dof_vector()
        mg.interpolate(l, v, vecs[0])
        vecs.insert(0, v)
        hl = []
        for h in hists[0]:
            t = ops[l - 1].initialize_dof_vector()
            mg.interpolate(l, t, h)
            hl.append(t)
        hists.insert(0, hl)
    for l, op in enumerate(ops):
        op.set_linearization_point(vecs[l])
        op.set_previous_solution(hists[l], w)
    torch.cuda.synchronize()
    mg.setup()
    return mg, ops


def vcycle_us(mg, n_dofs):
    b = torch.from_numpy(gi.rnd(7, n_dofs)).cuda()
    x = torch.zeros(n_dofs, dtype=torch.float64, device="cuda")
    return timed(lambda: mg.vcycle(x, b), REPS)


def main():
    d = gm.read_deck(os.path.join(gm.DECK_DIR, "input_hoffmann_3D_Re3900.json"))
    meshes = [d.mesh(r) for r in range(3)]
    vel, p, slip = d.boundary_descriptor()
    cmasks = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(meshes[-1].n_nodes, 3, d.u_max)
    hist = gi.history(u, params["order"])
    n0 = meshes[0].n_cells
    L = len(meshes) - 1
    # the redundant bottom of the agglomerated cycle: the global r0..r1 V-cycle
    u1 = gi.linearization_point(meshes[1].n_nodes, 3, d.u_max)
    gmg, gops = glsamd.build_gmg(meshes[:2], cmasks[:2], params, u1,
                                 gi.history(u1, params["order"]), w, precision="f32",
                                 smoothing_n_iterations=NS, coarse_n_iterations=COARSE)
    t_bottom = vcycle_us(gmg, meshes[1].n_dofs)
    n_r1 = meshes[1].n_dofs
    del gmg, gops
    rows = []
    for world in (1, 2, 4, 8):
        cb = glsdist.coarse_bounds(n0, world)
        parts = [glsdist.build_partitions(m, world, [b * (m.n_cells // n0) for b in cb])
                 for m in meshes]
        r = max(range(world), key=lambda q: parts[-1][q].n_cells)
        pf = parts[-1][r]
        u_f = u.reshape(-1, 4)[pf.local_nodes].ravel()
        h_f = [h.reshape(-1, 4)[pf.local_nodes].ravel() for h in hist]
        lms, lcm, ch = local_levels(meshes, cmasks, parts, r, list(range(L + 1)))
        mg, ops = multigrid(lms, lcm, ch, params, u_f, h_f, w, COARSE)
        t_vc = vcycle_us(mg, lms[-1].n_dofs)
        # the rank's r2 work alone (levels r1..r2, coarse solve = copy)
        mg2, ops2 = multigrid(lms[1:], lcm[1:], ch[1:], params, u_f, h_f, w, 0)
        t_top = vcycle_us(mg2, lms[-1].n_dofs)
        del mg2, ops2
        # FP64 local vmult and a GMRES(28) iteration on the rank's cells
        A = glsamd.NavierStokesOperator(lms[-1], lcm[-1], "f64")
        A.set_parameters(**params)
        A.set_linearization_point(u_f)
        A.set_previous_solution(h_f, w)
        src = A._dev(gi.src_vector(lms[-1].n_dofs))
        dst = A.initialize_dof_vector()
        t_vm = timed(lambda: A.vmult(dst, src), REPS)
        x = A.initialize_dof_vector()
        s = glsamd.LinearSolverGMRES(A, mg, n_max_iterations=28, relative_tolerance=1e-30,
                                     absolute_tolerance=0.0)

        def solve():
            try:
                s.solve(x, src)
            except glsamd.GlsError:
                pass
        t_gm = timed(solve, 3) / 28
        phases = 2 * (10 * L + (COARSE - 1)) + 2 * L   # partitioned cycle
        phases_agg = 2 * 10 + 1                         # r2 applies + one compress
        ar_bytes = n_r1 * 8                             # FP64 r1 right-hand side
        t_ar = (2 * (world - 1) / world * ar_bytes / (XGMI_GBS * 1e3) if world > 1 else 0.0)
        row = dict(world=world, rank=r, rank_cells=[p[r].n_cells for p in parts],
                   rank_dofs=lms[-1].n_dofs, vcycle_local_us=round(t_vc, 1),
                   r2_level_local_us=round(t_top, 1), bottom_r0_r1_global_us=round(t_bottom, 1),
                   vmult_f64_local_us=round(t_vm, 1), gmres_iteration_local_us=round(t_gm, 1),
                   halo_phases=phases if world > 1 else 0,
                   halo_phases_agglomerated=phases_agg if world > 1 else 0,
                   allreduce_r1_bytes=ar_bytes if world > 1 else 0,
                   allreduce_r1_us=round(t_ar, 1), allreduce_gbs_assumed=XGMI_GBS)
        proj = {}
        for eps in EPS_US:
            ex = (phases if world > 1 else 0) * eps
            exa = (phases_agg * eps + t_ar + 2 * eps) if world > 1 else 0.0
            proj[f"eps{eps:g}"] = dict(
                vcycle_us=round(t_vc + ex, 1),
                vcycle_agglomerated_us=round(t_top + t_bottom + exa, 1) if world > 1 else None)
        row["projection"] = proj
        rows.append(row)
        print(json.dumps(row), flush=True)
        del mg, ops, A, s
    print("\nworld  rank cells(r2)  local V-cycle  r2 level  + r0..r1 global  "
          "| projected V-cycle (eps 4.2 / 10 / 20 us per halo phase): partitioned ; agglomerated")
    for row in rows:
        pj = row["projection"]
        part = " / ".join(f"{pj[k]['vcycle_us']:7.1f}" for k in pj)
        agg = " / ".join("   -   " if pj[k]["vcycle_agglomerated_us"] is None else
                         f"{pj[k]['vcycle_agglomerated_us']:7.1f}" for k in pj)
        print(f"{row['world']:5d}  {row['rank_cells'][-1]:14d}  {row['vcycle_local_us']:12.1f}  "
              f"{row['r2_level_local_us']:8.1f}  {row['bottom_r0_r1_global_us']:15.1f}  | "
              f"{part} ; {agg}")


if __name__ == "__main__":
    main()
