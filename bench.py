#!/usr/bin/env python3
"""bench.py — vmult DoF/s + achieved HBM-roofline fraction of the matrix-free
GLS Navier–Stokes operator on MI355X (BASELINE.json metric).

Workload (N = 1): input_hoffmann_3D_Re3900.json — 3D flow past a cylinder,
Q2/Q2 (FESystem(FE_Q(2), 4)), QGauss(3), MappingQ2, 2 global refinements
(25,600 cells, 878,592 DoFs), Newton-Jacobian (increment-form) operator in
FP64, BDF2 with dt = 2.5e-4, synthetic inputs of SURVEY §8d.  One "step" =
one operator apply (vmult) on inputs already resident in HBM.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--nref R]
For N > 1 launch with torch.distributed.run (one rank per GPU); cells are
partitioned into contiguous x-slabs, ghost DoFs exchanged over RCCL.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))

import numpy as np  # noqa: E402

import glsinputs as gi  # noqa: E402
import glsmesh as gm  # noqa: E402

HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E spec (MI355X_MICROARCH.md)
DECK = "input_hoffmann_3D_Re3900.json"


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


PARITY_TOL = {"f64": 1e-12, "f32": 2e-5}  # relative l2 vs the oracle (tests/ use the same)


def make_oracle(case_mesh, cmask, params, weights, u_star, hist):
    """The CPU restatement (oracle/, TEST INFRASTRUCTURE) on the bench's own
    inputs: the checker of the headline result and the cpu_baseline leg."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    orc.set_threads(threads)
    om = orc.OracleMesh(case_mesh, cmask)
    o = orc.Oracle(om, **params)
    o.set_linearization_point(u_star)
    if params["order"] > 0:
        o.set_previous_solution(hist, weights)
    o._threads = threads
    o._mesh = om
    return o


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def cpu_baseline(o, src, n_dofs, budget_s=12.0):
    """SURVEY §8d CPU baseline: the cell-batched SIMD restatement of the same
    vmult (oracle/gls_cpu_batched.c: W = 8 cells per AVX-512 vector,
    MatrixFree-style per-batch tables and compressed geometry, coloured
    batches, OpenMP), 'port', timed on a bounded sample of whole vmults of
    the same mesh, on every host core this job may use (OMP_NUM_THREADS, the
    box's CPU share) and on 1 core.  Results checked against the scalar
    oracle before timing."""
    import oracle as orc

    def rate(b, budget):
        b.vmult(src)  # warm-up
        reps, t0 = 0, time.perf_counter()
        while True:
            b.vmult(src)
            reps += 1
            el = time.perf_counter() - t0
            if el > budget:
                return reps, el

    threads = o._threads
    b = orc.BatchedCPU(o, threads)
    chk = rel_l2(b.vmult(src), o.vmult(src))
    if not chk < 1e-12:
        raise RuntimeError(f"batched CPU baseline disagrees with the oracle ({chk:.1e})")
    reps, el = rate(b, 0.6 * budget_s)
    b1 = orc.BatchedCPU(o, 1)
    reps1, el1 = rate(b1, 0.4 * budget_s)
    return dict(value=n_dofs * reps / el, unit="DoF/s", cores=threads, kind="port",
                value_1core=n_dofs * reps1 / el1, cores_1=1,
                cpu_model=orc.cpu_model(), nproc=os.cpu_count(), isa=b.isa,
                sample=f"{reps} ({threads} threads) + {reps1} (1 thread) whole FP64 Newton "
                       f"vmults of the same Re3900 mesh ({n_dofs} DoFs): "
                       f"oracle/gls_cpu_batched.c ({b.isa}, 8 cells per vector, "
                       f"{b.n_colors} batch colours), {el:.1f} s + {el1:.1f} s; "
                       f"agrees with the scalar oracle to {chk:.1e}")


def _comp_get(comp, key, field):
    v = (comp or {}).get(key)
    return v.get(field) if isinstance(v, dict) else None


def _timed_vmults(op, dst, src, reps, flush=None):
    """Median per-vmult duration (ms) with HIP events on the launch stream
    (torch's current stream); `flush` runs between reps, outside the events."""
    import torch
    t = []
    for _ in range(reps):
        if flush is not None:
            flush()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        op.vmult(dst, src)
        e1.record()
        torch.cuda.synchronize()
        t.append(e0.elapsed_time(e1))
    return float(np.median(t))


def survey_bytes(op, td=True, cell_wise=False):
    """SURVEY §8d's algorithmic bytes of one vmult, the roofline's numerator:
    s 2N + s C nq n_tab + s [n_gen nq (dim^2+1) + n_cart (dim+1)] + 4 C nq,
    n_tab = the reference's per-q table values of the Newton vmult
    (operator_ns.h:120-132: delta_1, delta_2, U, grad U, grad P, and U_t with
    the time derivative; 20 in 3D).  The brick kernel streams fewer (T1 and h
    instead of grad P, U_t, delta_1/2: op.vmult_bytes()), so the bytes it
    moves are below this figure."""
    s = float(op.dtype.itemsize)
    dim, nq = op.dim, (op.degree + 1) ** op.dim
    n_tab = 2 + dim + dim * dim + dim + (dim if td else 0) - (2 if cell_wise else 0)
    n_gen, n_cart = op.geometry_counts()
    C = float(op.n_cells)
    b = s * 2.0 * op.m() + s * C * nq * n_tab + s * (n_gen * nq * (dim * dim + 1) +
                                                    n_cart * (dim + 1)) + 4.0 * C * nq
    return b + (s * 2.0 * C if cell_wise else 0.0)


def companions(d, mesh, cmask, params, weights, n_ref, hot_op, hot_dst, hot_src, reps=50):
    """The rest of SURVEY §8d's timing protocol, beside the headline line:
    cold (MALL flushed by a 1 GiB scratch read between reps) vs warm FP64
    at r2, the FP32 level operator (the smoother's hot path) on the same
    mesh, the HBM-bound r+1 mesh (Turek-3D size at r2 = 3) and the
    unstructured sphere deck at r3 (17.1 M DoFs, all geometry per q).  Medians of
    `reps` event-timed vmults after 5 warm-ups."""
    import torch
    import glsamd
    out = {}
    # cold = the operator's data out of the MALL (256 MB) and the L2s: a 1 GiB
    # READ between reps, which leaves clean lines of another buffer.  A 1 GiB
    # WRITE (the flush of rounds 1-6, kept as *_cold_write_flush) leaves dirty
    # lines whose write-back the timed vmult's own reads trigger: +16.6 us per
    # r2 vmult inside its events (profiles/r06/explore/cold_probe.txt)
    scratch = torch.zeros(1 << 30, dtype=torch.uint8, device="cuda")
    scratch_f32 = scratch.view(torch.float32)
    sink = torch.zeros((), dtype=torch.float32, device="cuda")
    flush = lambda: torch.sum(scratch_f32, dim=0, out=sink)  # noqa: E731
    flush_write = lambda: scratch.fill_(1)  # noqa: E731

    def line(op, dst, src, fl=None, prec="f64"):
        for _ in range(5):
            op.vmult(dst, src)
        ms = _timed_vmults(op, dst, src, reps, fl)
        b = survey_bytes(op)
        r = {"ms": ms, "dofs_per_s": op.m() / (ms * 1e-3), "algorithmic_bytes": b,
             "streamed_bytes": op.vmult_bytes(),
             "roofline_frac": b / (ms * 1e-3) / HBM_PEAK, "dtype": prec}
        if fl is None:
            # the same vmults back to back between two events (how the
            # headline and the smoother run them: no host sync per call)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(reps):
                op.vmult(dst, src)
            e1.record()
            torch.cuda.synchronize()
            mb = e0.elapsed_time(e1) / reps
            r["ms_back_to_back"] = mb
            r["roofline_frac_back_to_back"] = b / (mb * 1e-3) / HBM_PEAK
        return r

    out[f"r{n_ref}_f64_warm"] = line(hot_op, hot_dst, hot_src)
    out[f"r{n_ref}_f64_cold"] = line(hot_op, hot_dst, hot_src, flush)
    out[f"r{n_ref}_f64_cold"]["flush"] = "1 GiB read between reps"
    out[f"r{n_ref}_f64_cold_write_flush"] = line(hot_op, hot_dst, hot_src, flush_write)
    out[f"r{n_ref}_f64_cold_write_flush"]["flush"] = (
        "1 GiB write between reps (its dirty lines written back inside the timed vmult)")

    def build(m, cm, prec, dk=d, prm=params, w=weights):
        u_star = gi.linearization_point(m.n_nodes, m.dim, dk.u_max)
        op = glsamd.NavierStokesOperator(m, cm, prec)
        op.set_parameters(**prm)
        op.set_linearization_point(u_star)
        if prm["order"] > 0:
            op.set_previous_solution(gi.history(u_star, prm["order"]), w)
        src = op._dev(gi.src_vector(m.n_dofs))
        return op, op.initialize_dof_vector(), src

    op32, dst32, src32 = build(mesh, cmask, "f32")
    out[f"r{n_ref}_f32_level_warm"] = line(op32, dst32, src32, prec="f32")
    del op32, dst32, src32
    vel, p, slip = d.boundary_descriptor()
    m3 = d.mesh(n_ref + 1)
    op3, dst3, src3 = build(m3, m3.constraint_mask(vel, p, slip), "f64")
    out[f"r{n_ref + 1}_f64_warm"] = line(op3, dst3, src3)
    out[f"r{n_ref + 1}_f64_warm"]["cells"] = m3.n_cells
    del op3, dst3, src3
    # the unstructured sphere deck (all cells general geometry, order 0)
    ds = gm.read_deck(os.path.join(gm.DECK_DIR, "input_sphere_amg.json"))
    ms = ds.mesh()
    ps, ws = ds.operator_parameters(2.5e-4)
    ops_, dsts, srcs = build(ms, ms.constraint_mask(*ds.boundary_descriptor()), "f64", ds, ps,
                             ws)
    out[f"sphere_r{ds.n_refinements}_f64_warm"] = line(ops_, dsts, srcs)
    out[f"sphere_r{ds.n_refinements}_f64_warm"]["cells"] = ms.n_cells
    del ops_, dsts, srcs
    # a deal.II cell order: the headline mesh with its
    # cells shuffled and nodes renumbered by first touch, bricks discovered
    # by gls_op_create (brick = {-1,-1,-1}), beside the per-cell kernel
    # (brick = {0,0,0}) on the same shuffled mesh; parity checked in
    # tests/test_brick_discovery.py
    sm = gm.ShuffledMesh(mesh, seed=1)
    smask = sm.constraint_mask(vel, p, slip)
    for tag, brick in (("auto_bricks", None), ("per_cell", (0, 0, 0))):
        u_s = gi.linearization_point(sm.n_nodes, sm.dim, d.u_max)
        op_s = glsamd.NavierStokesOperator(sm, smask, "f64", brick=brick)
        op_s.set_parameters(**params)
        op_s.set_linearization_point(u_s)
        if params["order"] > 0:
            op_s.set_previous_solution(gi.history(u_s, params["order"]), weights)
        src_s = op_s._dev(gi.src_vector(sm.n_dofs))
        key = f"r{n_ref}_f64_shuffled_{tag}"
        out[key] = line(op_s, op_s.initialize_dof_vector(), src_s)
        out[key]["brick_shape"] = list(op_s.brick_shape)
        del op_s, src_s
    out.update(mg_companions(d, params, weights, n_ref))
    del scratch
    torch.cuda.empty_cache()
    out.update(amg_companions())
    torch.cuda.empty_cache()
    try:
        out.update(turek3d_mg_companion())
    except Exception as e:  # reported beside the headline, never fatal
        out["turek3d_mg_f32_direct"] = {"error": str(e)}
    torch.cuda.empty_cache()
    return out


def mg_companions(d, params, weights, n_ref, reps=20):
    """The preconditioner side of a GMRES iteration on
    the Re3900 hierarchy r0..r{n_ref}, FP32 levels: the multigrid setup
    (inverse diagonals + power-iteration relaxation factors, gls_mg_setup),
    one V-cycle (5 damped-Jacobi pre/post steps; coarse solve = 10
    relaxation sweeps, the substitute for the deck's Trilinos direct solver,
    DESIGN.md A16), and one full right-preconditioned GMRES iteration (V-cycle
    + FP64 vmult + delayed CGS2); event-timed medians."""
    import torch
    import glsamd
    meshes = [d.mesh(r) for r in range(n_ref + 1)]
    vel, p, slip = d.boundary_descriptor()
    cm = [m.constraint_mask(vel, p, slip) for m in meshes]
    u = gi.linearization_point(meshes[-1].n_nodes, meshes[-1].dim, d.u_max)
    hist = gi.history(u, params["order"])
    mg, mg_ops = glsamd.build_gmg(meshes, cm, params, u, hist, weights, precision="f32",
                                  coarse_n_iterations=10)
    setup = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mg.setup()
        torch.cuda.synchronize()
        setup.append((time.perf_counter() - t0) * 1e3)
    A = glsamd.NavierStokesOperator(meshes[-1], cm[-1], "f64")
    A.set_parameters(**params)
    A.set_linearization_point(u)
    if params["order"] > 0:
        A.set_previous_solution(hist, weights)
    b = A._dev(gi.src_vector(meshes[-1].n_dofs))
    x = A.initialize_dof_vector()

    def vcycles():
        for _ in range(3):
            mg.vcycle(x, b)
        torch.cuda.synchronize()
        t = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            mg.vcycle(x, b)
            e1.record()
            torch.cuda.synchronize()
            t.append(e0.elapsed_time(e1))
        return float(np.median(t))

    def gmres_iteration(m):
        # fixed 28 iterations (one restart cycle), wall time per iteration
        solver = glsamd.LinearSolverGMRES(A, m, n_max_iterations=28, relative_tolerance=1e-30,
                                          absolute_tolerance=0.0)
        times = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            try:
                solver.solve(x, b)
            except glsamd.GlsError:
                pass  # no convergence at tolerance 0 is the point: 28 iterations
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) / max(1, solver.last["n_iterations"]))
        return float(np.median(times)) * 1e3

    vc = vcycles()
    # resident smoothing launches / spin-bound waits per level (coarsest first)
    sweeps = [list(op.sweep_stats()) for op in mg_ops]
    # the deck's own coarse solver ("gmg coarse grid solver": "direct",
    # multigrid.cc:448-455): the assembled r0 operator's free-dof block
    # LU-factorised and inverted once in the setup (rocSOLVER getrf/getri),
    # one GEMV over the FP32-stored inverse per V-cycle
    lu = {}
    try:
        mg_lu, _ = glsamd.build_gmg(meshes, cm, params, u, hist, weights, precision="f32",
                                    coarse_n_iterations=-1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mg_lu.setup()
        torch.cuda.synchronize()
        lu["setup_ms"] = (time.perf_counter() - t0) * 1e3
        # the dense coarse setup's parts: free block assembled from the
        # element matrices (one launch + a scatter per cell colour), getrf, getri
        lu["coarse_setup"] = mg_lu.coarse_setup_times()
        for _ in range(3):
            mg_lu.vcycle(x, b)
        torch.cuda.synchronize()
        t = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            mg_lu.vcycle(x, b)
            e1.record()
            torch.cuda.synchronize()
            t.append(e0.elapsed_time(e1))
        lu["ms"] = float(np.median(t))
        lu["gmres_iteration_ms"] = gmres_iteration(mg_lu)
        lu["coarse_dofs"] = meshes[0].n_dofs
        lu["coarse_free_dofs"] = int(sum(((c >> k) & 1 == 0).sum() for c in [cm[0]]
                                         for k in range(4)))
        # the dense inverse's size after the static condensation of the
        # cells' interior dofs (one interior Q2 node per 3D cell, never
        # constrained): free dofs - cells x (dim + 1)
        lu["inverse_dofs"] = lu["coarse_free_dofs"] - meshes[0].n_cells * (meshes[0].dim + 1)
        lu["inverse_storage"] = "f32 (FP64 sums), free dofs only"
        y32 = torch.zeros_like(x)
        mg_lu.vcycle(y32, b)
        del mg_lu
        # the same with the FP64-stored inverse: time and the V-cycle's
        # relative difference to the default FP32-stored inverse
        os.environ["GLS_COARSE_INV_F32"] = "0"
        try:
            mg_lu, _ = glsamd.build_gmg(meshes, cm, params, u, hist, weights, precision="f32",
                                        coarse_n_iterations=-1)
            mg_lu.setup()
            for _ in range(3):
                mg_lu.vcycle(x, b)
            torch.cuda.synchronize()
            t = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                mg_lu.vcycle(x, b)
                e1.record()
                torch.cuda.synchronize()
                t.append(e0.elapsed_time(e1))
            y64 = torch.zeros_like(x)
            mg_lu.vcycle(y64, b)
            torch.cuda.synchronize()
            lu["ms_inv_f64"] = float(np.median(t))
            lu["inv_f32_rel_diff"] = float(torch.linalg.norm((y32 - y64).double()) /
                                           torch.linalg.norm(y64.double()))
            del mg_lu
        finally:
            os.environ.pop("GLS_COARSE_INV_F32")
    except Exception as e:  # reported, never fatal
        lu = {"error": str(e)}
    git = gmres_iteration(mg)
    return {f"r{n_ref}_mg_setup_f32": {"ms": float(np.median(setup)), "levels": n_ref + 1,
                                       "note": "gls_mg_setup: inverse diagonals (direct "
                                               "element-diagonal kernel) + power iteration "
                                               "(20 steps, device reductions), wall"},
            f"r{n_ref}_vcycle_f32_coarse_relax10": {"ms": vc, "levels": n_ref + 1,
                                                    "finest_dofs": meshes[-1].n_dofs,
                                                    "vcycles_per_s": 1e3 / vc,
                                                    "resident_sweeps_launches_timeouts": sweeps},
            f"r{n_ref}_vcycle_f32_coarse_direct_lu": lu,
            f"r{n_ref}_gmres_iteration": {"ms": git,
                                          "note": "V-cycle (coarse: 10 relaxation sweeps) + "
                                                  "FP64 vmult + delayed CGS2 + host Hessenberg "
                                                  "step, "
                                                  "wall clock; with the deck's direct coarse "
                                                  "solve: r{}_vcycle_f32_coarse_direct_lu."
                                                  "gmres_iteration_ms".format(n_ref)}}


def turek3d_mg_companion(reps=10):
    """Config 3's own multigrid at its configured size (input_turek_3D_Re100
    .json: GMG over r0..r3, 6.8 M DoFs on the finest level, the HBM-bound
    size; deck coarse solver "direct", not iterated): FP32 levels, setup,
    one V-cycle (event-timed median) and one right-preconditioned GMRES
    iteration with the FP64 vmult (wall, 28 iterations of one restart)."""
    import torch
    import glsamd
    d = gm.read_deck(os.path.join(gm.DECK_DIR, "input_turek_3D_Re100.json"))
    params, w = d.operator_parameters(2.5e-4)
    n_ref = d.n_refinements
    meshes = [d.mesh(r) for r in range(n_ref + 1)]
    vel, p, slip = d.boundary_descriptor()
    cm = [m.constraint_mask(vel, p, slip) for m in meshes]
    u = gi.linearization_point(meshes[-1].n_nodes, meshes[-1].dim, d.u_max)
    hist = gi.history(u, params["order"])
    mg, _ = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                             coarse_n_iterations=-1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mg.setup()
    torch.cuda.synchronize()
    setup_ms = (time.perf_counter() - t0) * 1e3
    A = glsamd.NavierStokesOperator(meshes[-1], cm[-1], "f64")
    A.set_parameters(**params)
    A.set_linearization_point(u)
    if params["order"] > 0:
        A.set_previous_solution(hist, w)
    b = A._dev(gi.src_vector(meshes[-1].n_dofs))
    x = A.initialize_dof_vector()
    for _ in range(3):
        mg.vcycle(x, b)
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        mg.vcycle(x, b)
        e1.record()
        torch.cuda.synchronize()
        t.append(e0.elapsed_time(e1))
    solver = glsamd.LinearSolverGMRES(A, mg, n_max_iterations=28, relative_tolerance=1e-30,
                                      absolute_tolerance=0.0)
    times = []
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        try:
            solver.solve(x, b)
        except glsamd.GlsError:
            pass  # 28 iterations at tolerance 0
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) / max(1, solver.last["n_iterations"]))
    return {f"turek3d_r{n_ref}_mg_f32_direct": {
        "levels": n_ref + 1, "finest_dofs": meshes[-1].n_dofs, "coarse_dofs": meshes[0].n_dofs,
        "setup_ms": setup_ms, "coarse_setup": mg.coarse_setup_times(),
        "vcycle_ms": float(np.median(t)), "gmres_iteration_ms": float(np.median(times)) * 1e3}}


def amg_companions(reps=5):
    """The AMG decks' coarse solver (multigrid.cc:372-433,
    491-530): FE_Q_iso_Q1 coarse level, "gmg coarse grid iterate" (GMRES to
    1e-4) preconditioned by the smoothed-aggregation AMG (gls_amg_*, the
    substitute for Trilinos ML) against the same coarse GMRES preconditioned
    by 10 relaxation sweeps: coarse GMRES iterations, wall ms per V-cycle,
    AMG setup and hierarchy, on the sphere (r3, its configured size) and the
    stationary Re20 deck (r2).  The Re20 deck's saddle-point coarse level
    diverges under Jacobi sweeps: no relaxation line there."""
    import torch
    import glsamd
    out = {}
    for name, n_ref, relax in (("input_sphere_amg.json", 3, True),
                               ("input_turek_2D_Re20_stat.json", 2, False)):
        d = gm.read_deck(os.path.join(gm.DECK_DIR, name))
        params, w = d.operator_parameters(2.5e-4)
        meshes = [d.mesh(r) for r in range(n_ref + 1)]
        vel, p, slip = d.boundary_descriptor()
        cm = [m.constraint_mask(vel, p, slip) for m in meshes]
        u = gi.linearization_point(meshes[-1].n_nodes, meshes[-1].dim, d.u_max)
        hist = gi.history(u, params["order"])
        b = torch.from_numpy(gi.src_vector(meshes[-1].n_dofs)).cuda()
        x = torch.zeros_like(b)
        line = {"finest_dofs": meshes[-1].n_dofs, "levels": n_ref + 1}
        # the AMG with deal.II's "smoother: Chebyshev alpha" 10 (the default)
        # and with ML's own default 30
        # the coarse iteration count per AMG level count (a smaller "coarse:
        # max size" forces a third level) and with the near-null space split
        # per component (dim + 1 constant modes, node blocks: what
        # extract_constant_modes hands ML when the deck does not ask for the
        # default parameters), to show where the AMG's weakness comes from
        variants = [("amg", dict(coarse_amg=d.amg_parameters())),
                    ("amg_alpha30", dict(coarse_amg=dict(d.amg_parameters(),
                                                         chebyshev_alpha=30.0))),
                    ("amg_3levels", dict(coarse_amg=dict(d.amg_parameters(),
                                                         coarse_max_size=100))),
                    ("amg_component_modes", dict(coarse_amg=dict(d.amg_parameters(),
                                                                 block_size=d.dim + 1)))]
        if relax:
            variants.append(("relax10", dict(coarse_n_iterations=10)))
        for key, kw in variants:
            try:
                mg, _ = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                                         coarse_iso_q1=True, coarse_iterate=True,
                                         coarse_reltol=1e-4, coarse_maxiter=2000, **kw)
                mg.vcycle(x, b)
                torch.cuda.synchronize()
                t = []
                for _ in range(reps):
                    t0 = time.perf_counter()
                    mg.vcycle(x, b)
                    torch.cuda.synchronize()
                    t.append((time.perf_counter() - t0) * 1e3)
                it, conv = mg.coarse_statistics()
                r = {"vcycle_ms": float(np.median(t)), "coarse_gmres_iterations": it,
                     "converged": conv, "coarse_dofs": meshes[0].n_dofs}
                if key.startswith("amg"):
                    info, setup_ms = mg.coarse_amg()
                    r.update(amg_setup_ms=setup_ms, amg_levels=info["levels"],
                             amg_sizes=info["sizes"], amg_nnz=info["nnz"])
                line[key] = r
                del mg
            except Exception as e:  # reported, never fatal
                line[key] = {"error": str(e)}
        out[f"{d.simulation}_{'2d' if d.dim == 2 else '3d'}_r{n_ref}_coarse_gmres"] = line
    return out


def dist_size_companion(d, params, weights, n_ref, dist, rank, world, reps=30):
    """Multi-GPU beside the strong-scaled headline: the same deck one
    refinement finer (r{n_ref+1}, 8x the cells: the HBM-bound size where the
    halo exchange no longer dominates), partitioned the same
    way, FP64 vmult over RCCL; barrier-bracketed wall time per vmult, max
    over ranks.  B_tab per vmult over the aggregate HBM peak of the ranks."""
    import torch
    import glsdist
    m = d.mesh(n_ref + 1)
    vel, p, slip = d.boundary_descriptor()
    cm = m.constraint_mask(vel, p, slip)
    u = gi.linearization_point(m.n_nodes, m.dim, d.u_max)
    hist = gi.history(u, params["order"])
    A = glsdist.DistributedOperator(m, cm, "f64", dist, rank, world)
    A.setup(params, u, hist, weights)
    src = A.scatter_global(gi.src_vector(m.n_dofs))
    dst = A.new_vector()
    for _ in range(3):
        A.vmult(dst, src)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        A.vmult(dst, src)
    torch.cuda.synchronize()
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms = float(t.item()) / reps * 1e3
    b = torch.tensor([survey_bytes(A.op)], dtype=torch.float64, device="cuda")
    dist.all_reduce(b)  # the ranks' local algorithmic bytes (ghost cells counted once each)
    return {f"r{n_ref + 1}_f64_dist": {
        "ms": ms, "dofs": m.n_dofs, "cells": m.n_cells, "dofs_per_s": m.n_dofs / (ms * 1e-3),
        "n_gpus": world, "algorithmic_bytes_all_ranks": float(b.item()),
        "roofline_frac_aggregate": float(b.item()) / (ms * 1e-3) / (HBM_PEAK * world),
        "cells_per_gpu": m.n_cells / world,
        # at 8 ranks r{n+1} gives every GPU the single-GPU headline's cell
        # count: the weak-scaling point of SURVEY §8e beside the strong-scaled
        # headline (8x the DoFs in the same per-GPU work)
        "weak_scaling_point": world == 8,
        "note": "DistributedOperator (native RCCL halo import overlapped with interior bricks, "
                "export-add), wall clock max over ranks"}}


def dist_gmres_companion(d, params, weights, n_ref, dist, rank, world, reps=10):
    """The whole GMRES iteration on N GPUs: the partitioned
    multigrid (glsdist.DistributedMultigrid: FP32 levels on the same
    coarse-cell partition, halo exchanges around the transfers, all-reduced
    power-iteration dots; coarse solve 10 relaxation sweeps) preconditioning
    right GMRES on the FP64 distributed operator with all-reduced CGS2 dots.
    Wall times, barrier-bracketed, max over ranks: setup, one V-cycle, one
    GMRES iteration (28 iterations = one restart cycle, tolerance 0)."""
    import torch
    import glsdist
    meshes = [d.mesh(r) for r in range(n_ref + 1)]
    vel, p, slip = d.boundary_descriptor()
    cm = [m.constraint_mask(vel, p, slip) for m in meshes]
    u = gi.linearization_point(meshes[-1].n_nodes, meshes[-1].dim, d.u_max)
    hist = gi.history(u, params["order"])
    dmg = glsdist.DistributedMultigrid(meshes, cm, "f32", dist, rank, world,
                                       coarse_n_iterations=10)
    top = dmg.levels[-1]
    dmg.set_linearization_point(params, top.scatter_global(u),
                                [top.scatter_global(h) for h in hist], weights)
    A = dmg.fine_operator("f64")
    A.setup(params, u, hist, weights)
    b = A.scatter_global(gi.src_vector(meshes[-1].n_dofs))
    x = A.new_vector()

    def wall(fn, n):
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    dmg.setup()
    t_setup = wall(dmg.setup, 3)
    dmg.vmult(x, b)
    t_vc = wall(lambda: dmg.vmult(x, b), reps)

    def gmres():
        try:
            glsdist.gmres_solve(lambda dst, src: A.vmult(dst, src),
                                lambda dst, src: dmg.vmult(dst, src), b, x,
                                A.r.n_owned_dofs, lambda t: dist.all_reduce(t),
                                max_iterations=28, relative_tolerance=0.0,
                                absolute_tolerance=0.0)
        except RuntimeError:
            pass  # tolerance 0: exactly 28 iterations

    gmres()  # warm-up: the Krylov basis allocation stays in torch's cache
    its = 2 * 28
    t_gm = wall(gmres, 2)
    out = {f"r{n_ref}_dist_mg_setup_f32": {"ms": t_setup / 3 * 1e3, "levels": n_ref + 1},
           f"r{n_ref}_dist_vcycle_f32_coarse_relax10": {"ms": t_vc / reps * 1e3},
           f"r{n_ref}_dist_gmres_iteration": {
               "ms": t_gm / its * 1e3, "n_gpus": world,
               "note": "glsdist.DistributedMultigrid V-cycle + FP64 distributed vmult + "
                       "all-reduced CGS2, host-driven, wall clock max over ranks"}}
    # the same through the native team calls (gls_dist_mg_* V-cycle and
    # gls_dist_gmres_solve: one C-ABI call per V-cycle / solve per rank)
    try:
        import glsamd
        nmg = dmg.native(params, u, hist, weights)
        fine_h = A.native
        glsamd.PartitionedMultigrid.vcycle([nmg], [x], [b])
        t_nvc = wall(lambda: glsamd.PartitionedMultigrid.vcycle([nmg], [x], [b]), reps)

        def ngmres():
            try:
                glsamd.dist_gmres_solve([fine_h], [nmg], [x], [b], n_max_iterations=28,
                                        relative_tolerance=0.0, absolute_tolerance=0.0)
            except glsamd.GlsError:
                pass  # tolerance 0: exactly 28 iterations
        ngmres()
        t_ngm = wall(ngmres, 2)
        out[f"r{n_ref}_dist_native_vcycle_f32_coarse_relax10"] = {"ms": t_nvc / reps * 1e3}
        out[f"r{n_ref}_dist_native_gmres_iteration"] = {
            "ms": t_ngm / its * 1e3, "n_gpus": world,
            "note": "gls_dist_mg_vcycle + gls_dist_gmres_solve (native team calls, "
                    "RCCL all-reduced CGS2), wall clock max over ranks"}
        # level agglomeration: r0, r1 single-domain on every rank (one
        # all-reduce of the r1 right-hand side), r2 partitioned
        if n_ref >= 2:
            amg_ = dmg.native(params, u, hist, weights, redundant_levels=n_ref - 1)
            glsamd.PartitionedMultigrid.vcycle([amg_], [x], [b])
            t_avc = wall(lambda: glsamd.PartitionedMultigrid.vcycle([amg_], [x], [b]), reps)

            def agmres():
                try:
                    glsamd.dist_gmres_solve([fine_h], [amg_], [x], [b], n_max_iterations=28,
                                            relative_tolerance=0.0, absolute_tolerance=0.0)
                except glsamd.GlsError:
                    pass
            agmres()
            t_agm = wall(agmres, 2)
            out[f"r{n_ref}_dist_native_vcycle_f32_agglomerated"] = {
                "ms": t_avc / reps * 1e3, "redundant_levels": n_ref - 1}
            out[f"r{n_ref}_dist_native_gmres_iteration_agglomerated"] = {
                "ms": t_agm / its * 1e3, "n_gpus": world}
    except Exception as e:  # reported, never fatal
        out[f"r{n_ref}_dist_native_gmres_iteration"] = {"error": str(e)}
    return out


def launch_ranks(args, argv):
    """`bench.py --gpus N` without a launcher (WORLD_SIZE unset, N > 1): start
    N ranks as ONE child process `python -m torch.distributed.run
    --nproc-per-node N ... bench.py <same arguments>` (the reference's
    `mpirun -np N`, input_hoffmann_2D_ReInf_3D.sh:8), relay rank 0's JSON line
    and exit with the child's status.  Called before anything touches the GPU;
    never exec's (the child is a subprocess).  A line whose n_gpus differs
    from N fails the run."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", str(max(1, min(16, (os.cpu_count() or 1) // args.gpus))))
    log(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}")
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip().startswith("{")]
    if not lines:
        log(f"[bench] launcher: no JSON line from the ranks (exit {p.returncode})")
        return p.returncode or 5
    line = lines[-1]
    try:
        n = json.loads(line).get("n_gpus")
    except ValueError:
        n = None
    print(line, flush=True)
    if n != args.gpus:
        log(f"[bench] launcher: n_gpus {n} in the line differs from --gpus {args.gpus}")
        return p.returncode or 6
    return p.returncode


def dry_run(args, out_fd):
    """--dry-run: the launch plumbing without the GPU (CPU tests): every rank
    joins a gloo group, checks WORLD_SIZE == --gpus, all-reduces its rank, and
    rank 0 prints a JSON line of the bench's shape with n_gpus = world."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
        t = torch.tensor([float(rank)])
        dist.all_reduce(t)
        assert float(t) == world * (world - 1) / 2
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"metric": "dry-run", "value": 0.0, "unit": "DoF/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "dry_run": True}),
              file=out_fd, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--dry-run", action="store_true",
                    help="launch plumbing only (gloo, no GPU): the CPU test of --gpus N")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--settle-ms", type=float, default=200.0,
                    help="untimed back-to-back steps for about this long before the W "
                         "warm-up steps, so the timed region runs at the sustained clock "
                         "(0: off; reported as 'settle' in the line)")
    ap.add_argument("--nref", type=int, default=None)
    ap.add_argument("--precision", default="f64")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-companions", action="store_true",
                    help="skip the cold / FP32-level / r+1 companion lines")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--brick", default=None,
                    help="cells per brick 'bx,by,bz' (a sub-brick of the mesh order)")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the oracle check of the headline result (profiling runs)")
    ap.add_argument("--gmres-iteration", action="store_true",
                    help="multi-GPU (or GLS_BENCH_DIST=1): also time the partitioned "
                         "multigrid + GMRES iteration (reported beside the headline)")
    ap.add_argument("--allow-p2p-fallback", action="store_true",
                    help="(default since round 6; kept for old command lines)")
    ap.add_argument("--strict-native", action="store_true",
                    help="multi-GPU: exit 4 when the native RCCL vmult disagrees with the "
                         "torch P2P path (or fails) instead of timing the P2P path")
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and (world > 1 or args.gpus > 1):
        log(f"[bench] WORLD_SIZE {world} differs from --gpus {args.gpus}")
        sys.exit(2)
    # stdout carries exactly one JSON line: everything else the process or
    # its libraries write to fd 1 (RCCL's version banner, ...) goes to stderr
    out_fd = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    if args.dry_run:
        dry_run(args, out_fd)
        return

    import torch
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dist = None
    # GLS_BENCH_DIST=1: the partitioned path at world 1 too (a rehearsal of
    # the multi-GPU code path on a one-GPU box)
    use_dist = world > 1 or os.environ.get("GLS_BENCH_DIST") == "1"
    if use_dist:
        import torch.distributed as dist
        if "RANK" not in os.environ:  # GLS_BENCH_DIST=1 without a launcher
            import socket
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
            os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(port))
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    import glsamd
    d = gm.read_deck(os.path.join(gm.DECK_DIR, DECK))
    n_ref = d.n_refinements if args.nref is None else args.nref
    t0 = time.time()
    mesh = d.mesh(n_ref)
    vel, p, slip = d.boundary_descriptor()
    cmask = mesh.constraint_mask(vel, p, slip)
    params, weights = d.operator_parameters(2.5e-4)
    n_dofs = mesh.n_dofs
    src_h = gi.src_vector(n_dofs)
    u_star = gi.linearization_point(mesh.n_nodes, mesh.dim, d.u_max)
    hist = gi.history(u_star, params["order"])
    log(f"[bench] mesh {mesh.n_cells} cells, {n_dofs} DoFs ({time.time() - t0:.1f}s)")

    region_events = False
    native_check = None
    if use_dist:
        import glsdist
        runner = glsdist.DistributedOperator(mesh, cmask, args.precision, dist, rank, world)
        runner.setup(params, u_star, hist, weights)
        src = runner.scatter_global(src_h)
        dst = runner.new_vector()
        # cross-check the native RCCL path (gls_dist_vmult) against the
        # torch point-to-point exchange around the same local operator once;
        # on a mismatch every rank falls back to the latter (reported)
        # (RCCL with real peers has not run before a multi-GPU lease: a native
        # failure or mismatch is reported in the line and, unless
        # --strict-native, the same kernels are timed with the torch P2P
        # exchange, labelled in "exchange")
        exchange = "rccl-native, overlapped with the interior bricks"
        ref = runner.new_vector()
        runner.vmult_p2p(ref, src.clone())
        s2 = src.clone()
        s2[runner.r.n_owned_dofs:].zero_()
        native_error = None
        try:
            runner.vmult(dst, s2)
            torch.cuda.synchronize()
        except Exception as e:  # the native exchange failed: no common result
            native_error = f"{type(e).__name__}: {e}"
            log(f"[bench] native partitioned vmult failed: {native_error}")
            dst.fill_(float("nan"))
        n = runner.r.n_owned_dofs
        err = torch.tensor([float((dst[:n] - ref[:n]).norm()), float(ref[:n].norm())],
                           dtype=torch.float64, device="cuda")
        dist.all_reduce(err)
        rel = float(err[0]) / max(float(err[1]), 1e-300)
        log(f"[bench] native vs p2p partitioned vmult: rel err {rel:.2e}")
        native_check = {"rel_l2_vs_torch_p2p": rel, "ok": bool(rel < 1e-12)}
        if native_error:
            native_check["error"] = native_error
        if not rel < 1e-12:
            if args.strict_native:
                if rank == 0:
                    print(json.dumps({"error": "native RCCL partitioned vmult disagrees with "
                                               "the torch P2P path", "rel_l2": rel}),
                          file=out_fd, flush=True)
                dist.barrier()
                dist.destroy_process_group()
                sys.exit(4)
            runner.native = None
            exchange = f"torch-p2p (native check failed: rel {rel:.1e})"
        apply_fn = lambda: runner.vmult(dst, src)  # noqa: E731
        local_cells = runner.n_local_cells
        op = runner.op

        def kernel_fn(ev0, ev1):
            # rank-local cell loop (k_brick + k_shared_reduce), no exchange
            ev0.record()
            op.vmult(ref, src)
            ev1.record()
    else:
        brick = tuple(int(x) for x in args.brick.split(",")) if args.brick else None
        op = glsamd.NavierStokesOperator(mesh, cmask, args.precision, brick=brick)
        op.set_parameters(**params)
        op.set_linearization_point(u_star)
        if params["order"] > 0:
            op.set_previous_solution(hist, weights)
        src = op._dev(src_h)
        dst = op.initialize_dof_vector()
        local_cells = op.n_cells
        exchange = None

        def apply_fn():
            op.vmult(dst, src)

        def kernel_fn(ev0, ev1):
            # the vmult is k_brick (dominant) + k_shared_reduce on one stream
            ev0.record()
            op.vmult(dst, src)
            ev1.record()
        # one step is exactly the vmult's two launches: the events around the
        # timed region give their average duration
        region_events = True

    torch.cuda.synchronize()
    # clock settle, untimed, before the W warm-up steps: after the setup's
    # seconds of GPU idleness the first ~20 ms of vmults run at a lower clock
    # (profiles/r06/explore/clock_probe.txt: 38.6 -> 34.2 us per step over 600
    # back-to-back vmults after 3 s idle; this loop's W + K pattern 36.1-36.5
    # us with no settle, 33.1-33.8 us after 100 ms of vmults).  A solver runs
    # the operator at the sustained clock.  Every rank runs the same number of
    # steps (the partitioned step is collective): ten timed steps, then the
    # count for settle_ms from the slowest rank.
    settle = None
    if args.settle_ms > 0:
        t_settle = time.perf_counter()
        for _ in range(10):
            apply_fn()
        torch.cuda.synchronize()
        per = torch.tensor([(time.perf_counter() - t_settle) / 10], dtype=torch.float64,
                           device="cuda")
        if dist is not None:
            dist.all_reduce(per, op=dist.ReduceOp.MAX)
        n_settle = 10 + max(0, int(args.settle_ms * 1e-3 / max(float(per.item()), 1e-6)) - 10)
        for _ in range(n_settle - 10):
            apply_fn()
        torch.cuda.synchronize()
        settle = {"steps": n_settle, "ms": (time.perf_counter() - t_settle) * 1e3,
                  "target_ms": args.settle_ms}
    for _ in range(args.warmup):
        apply_fn()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    # region events (instrumentation: created and the opening one enqueued
    # before the clock starts -- creating and recording them inside it cost
    # ~50 us of host time per region, profiles/r06/explore/sync_probe.txt).
    # ev_region[0]: stamped at once (idle GPU), so [0]..[2] also holds the
    # first step's launch from an idle queue; ev_region[1]: after step 1, when
    # the host is ahead of the GPU, so [1]..[2] holds steps 2..K back to back
    # -- the kernels' own average duration, what rocprofv3 averages
    if region_events:
        ev_region = tuple(torch.cuda.Event(enable_timing=True) for _ in range(3))
        ev_region[0].record()
    t_start = time.perf_counter()
    for i in range(args.steps):
        apply_fn()
        if region_events and i == 0:
            ev_region[1].record()
    if region_events:
        ev_region[2].record()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t_start
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ms = el / args.steps * 1e3
    value = n_dofs * args.steps / el

    # average duration of the dominant kernel pair (k_brick + reduce), HIP
    # events on the stream it is launched on (torch's current stream): single
    # GPU, the region events after step 1 / (K - 1) (the vmults back to back,
    # as rocprofv3 sees them); partitioned, the rank-local cell loop between its
    # own events.  kernel_ms_event_pairs: one event pair around each of K more
    # vmults (the event packets between the launches add ~3 us per vmult)
    kernel_ms = kernel_ms_pairs = None
    if kernel_fn is not None:
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        for e0, e1 in evs:
            kernel_fn(e0, e1)
        torch.cuda.synchronize()
        kernel_ms_pairs = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))
        kernel_ms = kernel_ms_pairs
    kernel_ms_region = None
    if region_events:
        kernel_ms_region = ev_region[0].elapsed_time(ev_region[2]) / args.steps
        kernel_ms = (ev_region[1].elapsed_time(ev_region[2]) / (args.steps - 1)
                     if args.steps > 1 else kernel_ms_region)

    dist_comp = None
    if use_dist and not args.no_companions:
        try:  # reported beside the headline, never fatal (failures are symmetric: same
            # mesh and code on every rank)
            dist_comp = dist_size_companion(d, params, weights, n_ref, dist, rank, world)
        except Exception as e:
            dist_comp = {f"r{n_ref + 1}_f64_dist": {"error": str(e)}}
        log(f"[bench] distributed r{n_ref + 1}: {dist_comp}")
    if use_dist and args.gmres_iteration:
        g = dist_gmres_companion(d, params, weights, n_ref, dist, rank, world)
        dist_comp = dict(dist_comp or {}, **g)
        log(f"[bench] distributed GMRES iteration: {g}")
    bytes_per_vmult = survey_bytes(op)
    n_gen, n_cart = op.geometry_counts()
    # parity of the timed result: the headline dst (FP64) against the oracle
    # on the same inputs (and the FP32 level operator at N = 1); a result
    # outside the tolerance fails the run
    got = None
    if not args.no_parity:
        apply_fn()
        torch.cuda.synchronize()
        got = (runner.gather_global(dst) if use_dist else dst).double().cpu().numpy()
    o = None
    if rank == 0 and (not args.no_parity or not args.no_cpu_baseline):
        o = make_oracle(mesh, cmask, params, weights, u_star, hist)
    parity = None
    if rank == 0 and not args.no_parity:
        ref = o.vmult(src_h)
        parity = {"rel_l2_" + args.precision: rel_l2(got, ref),
                  "tol_" + args.precision: PARITY_TOL[args.precision],
                  "oracle": "oracle/gls_oracle.c on the same mesh and inputs"}
        if world == 1 and not use_dist and args.precision == "f64":
            op32 = glsamd.NavierStokesOperator(mesh, cmask, "f32")
            op32.set_parameters(**params)
            op32.set_linearization_point(u_star)
            if params["order"] > 0:
                op32.set_previous_solution(hist, weights)
            d32 = op32.initialize_dof_vector()
            op32.vmult(d32, op32._dev(src_h))
            torch.cuda.synchronize()
            parity["rel_l2_f32"] = rel_l2(d32.double().cpu().numpy(), ref)
            parity["tol_f32"] = PARITY_TOL["f32"]
            del op32, d32
        parity["ok"] = all(parity["rel_l2_" + p] < parity["tol_" + p]
                           for p in ("f64", "f32") if "rel_l2_" + p in parity)
        log(f"[bench] parity vs oracle: {parity}")
    out = None
    if rank == 0:
        if kernel_ms is None:
            kernel_ms = ms
        achieved = bytes_per_vmult / (kernel_ms * 1e-3)
        # HBM bytes per vmult from the committed rocprofv3 PMC passes of this
        # workload (scripts/pmc.sh + scripts/pmc_summary.py), when they match
        traffic = None
        # the newest round's PMC record of the headline kernel pair
        tf = os.environ.get("GLS_TRAFFIC_JSON")
        if tf is None:
            for rnd in ("r06", "r05"):
                tf = os.path.join(ROOT, "profiles", rnd, "pmc_r2", "traffic.json")
                if os.path.exists(tf):
                    break
        if tf and os.path.exists(tf) and world == 1:
            with open(tf) as f:
                tj = json.load(f)
            wl = tj.get("workload", {})
            if wl.get("nref") == n_ref and wl.get("precision") == args.precision:
                traffic = tj.get("bytes_per_launch")
        comp = None
        if not args.no_companions and world == 1 and kernel_fn is not None and not use_dist:
            try:
                comp = companions(d, mesh, cmask, params, weights, n_ref, op, dst, src)
            except Exception as e:  # reported beside the headline, never fatal
                comp = {"error": str(e)}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(o, src_h, n_dofs, args.cpu_budget)
            except Exception as e:  # baseline is reported, never fatal
                cpu = dict(value=None, unit="DoF/s", cores=0, kind="port", sample=f"failed: {e}")
        out = {
            "metric": "vmult DoF/s (3D cylinder Re=3900 Q2, FP64 Newton-Jacobian GLS operator)",
            "value": value,
            "unit": "DoF/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            # untimed steps before the warm-up (the sustained clock, see above)
            "settle": settle,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64" if args.precision == "f64" else "f32",
            "data": "synthetic (SURVEY §8d splitmix64 inputs on the generated cylinder mesh)",
            "config": {"workload": f"{DECK} r{n_ref}: {mesh.n_cells} cells, {n_dofs} DoFs, "
                                   f"Q2/Q2, MappingQ2, BDF2, increment form",
                       "cells": mesh.n_cells, "dofs": n_dofs, "cells_per_gpu": local_cells,
                       "general_geometry_cells": n_gen, "cartesian_cells": n_cart,
                       "brick_shape": list(op.brick_shape) if hasattr(op, "brick_shape") else None,
                       "parallelism": f"cells x-slab partitioned over {world} GPU(s)"
                                      + (f", ghost exchange {exchange}" if exchange else "")},
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK, "traffic": traffic,
                         "kernel": "vmult = gls::k_brick<3,2,double,MODE_NEWTON> + "
                                   "gls::k_shared_reduce_cls (both inside the events)",
                         "kernel_ms": kernel_ms, "kernel_ms_event_pairs": kernel_ms_pairs,
                         # the whole region / K (first launch from an idle queue included)
                         "kernel_ms_region": kernel_ms_region,
                         "algorithmic_bytes": bytes_per_vmult,
                         "streamed_bytes": op.vmult_bytes(),
                         # the same launch time against what the kernel reads
                         # (16 instead of SURVEY's 20 table values per q)
                         "frac_streamed": op.vmult_bytes() / (kernel_ms * 1e-3) / HBM_PEAK,
                         # SURVEY §8d's cold r2 figure (MALL flushed by a 1 GiB
                         # read between vmults, one synchronize per call; the
                         # warm 133 MB working set fits the 256 MB MALL), the
                         # rounds-1-6 write flush beside it, and the HBM-bound
                         # r+1 mesh back to back, from the companions below
                         # (null without them)
                         "frac_cold": _comp_get(comp, f"r{n_ref}_f64_cold", "roofline_frac"),
                         "frac_cold_write_flush": _comp_get(comp, f"r{n_ref}_f64_cold_write_flush",
                                                            "roofline_frac"),
                         "frac_r3": _comp_get(comp, f"r{n_ref + 1}_f64_warm",
                                              "roofline_frac_back_to_back")},
            "cpu_baseline": cpu,
            "parity": parity,
            "native_exchange_check": native_check,
            "companions": comp if dist_comp is None else dict(comp or {}, **dist_comp),
        }
        print(json.dumps(out), file=out_fd, flush=True)
    ok = parity is None or parity["ok"]
    if dist is not None:
        t = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64, device="cuda")
        dist.all_reduce(t)
        ok = float(t.item()) == 0.0
        dist.barrier()
        dist.destroy_process_group()
    if not ok:
        log("[bench] FAILED: result outside the parity tolerance")
        sys.exit(3)


if __name__ == "__main__":
    main()
