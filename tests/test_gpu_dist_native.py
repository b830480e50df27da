"""The native partitioned multigrid and GMRES behind the C-ABI
(gls_dist_mg_*, gls_dist_gmres_solve; csrc/dist_mg.hip),
run as in-process groups of 2 and 4 partitions on one GPU (the same team
calls an RCCL rank makes with n = 1) against the single-domain GPU
multigrid and GMRES on the same hierarchy.

FP64 levels: the V-cycle agrees with the single-domain one to 1e-10 (only
the summation order of partial sums across the partition differs); FP32
levels to 1e-5 (FP32 round-off of the reordered sums).  GMRES: the same
iteration count (+-1) and solution to 1e-8."""
import numpy as np
import pytest

import glsinputs as gi
from helpers import deck, rel_err

pytestmark = pytest.mark.gpu


def _hierarchy(n_ref=1):
    d = deck("input_hoffmann_3D_Re3900.json")
    meshes = [d.mesh(r) for r in range(n_ref + 1)]
    vel, p, slip = d.boundary_descriptor()
    cm = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(meshes[-1].n_nodes, 3, d.u_max)
    hist = gi.history(u, params["order"])
    return meshes, cm, params, w, u, hist


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("prec,coarse,n_ref", [("f64", 10, 1), ("f64", -1, 1), ("f32", 10, 1),
                                               # the production setup: FP32 levels with the
                                               # redundant direct coarse solve, 2 and 3 levels
                                               ("f32", -1, 1), ("f32", -1, 2)])
def test_native_group_vcycle(world, prec, coarse, n_ref):
    import torch
    import glsamd
    import glsdist
    meshes, cm, params, w, u, hist = _hierarchy(n_ref)
    ref, _ = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision=prec,
                              coarse_n_iterations=coarse)
    g = glsdist.NativeGroupMultigrid(meshes, cm, world, precision=prec,
                                     coarse_n_iterations=coarse)
    g.setup(params, u, hist, w)
    for l in range(len(meshes)):
        wd, lam = g.mg[0].relaxation(l)
        wr, lr = ref.relaxation(l)
        assert abs(wd - wr) <= 1e-6 * abs(wr), (l, wd, wr)
    b = gi.rnd(11, meshes[-1].n_dofs)
    bs = g.scatter(b)
    xs = [torch.zeros_like(x) for x in bs]
    g.vcycle(xs, bs)
    src = torch.from_numpy(b).cuda()
    dst = torch.zeros_like(src)
    ref.vcycle(dst, src)
    torch.cuda.synchronize()
    err = rel_err(g.gather(xs).cpu().numpy(), dst.cpu().numpy())
    print(f"world {world} {prec} coarse {coarse} levels {n_ref + 1}: partitioned vs "
          f"single-domain V-cycle {err:.2e}")
    assert err < (1e-10 if prec == "f64" else 1e-5)


@pytest.mark.parametrize("world", [2, 4])
def test_native_group_gmres(world):
    import torch
    import glsamd
    import glsdist
    meshes, cm, params, w, u, hist = _hierarchy(1)
    mg, _ = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f64",
                             coarse_n_iterations=-1)
    A = glsamd.NavierStokesOperator(meshes[-1], cm[-1], "f64")
    A.set_parameters(**params)
    A.set_linearization_point(u)
    A.set_previous_solution(hist, w)
    b = gi.rnd(12, meshes[-1].n_dofs)
    src = torch.from_numpy(b).cuda()
    x_ref = torch.zeros_like(src)
    solver = glsamd.LinearSolverGMRES(A, mg, relative_tolerance=1e-8, absolute_tolerance=0.0)
    solver.solve(x_ref, src)
    it_ref = solver.last["n_iterations"]
    g = glsdist.NativeGroupMultigrid(meshes, cm, world, precision="f64", coarse_n_iterations=-1)
    g.setup(params, u, hist, w)
    bs = g.scatter(b)
    xs = [torch.zeros_like(x) for x in bs]
    res = g.gmres(xs, bs, relative_tolerance=1e-8, absolute_tolerance=0.0)
    torch.cuda.synchronize()
    err = rel_err(g.gather(xs).cpu().numpy(), x_ref.cpu().numpy())
    print(f"world {world}: GMRES {res['n_iterations']} vs {it_ref} iterations, x rel diff {err:.2e}")
    assert res["converged"] and abs(res["n_iterations"] - it_ref) <= 1
    assert err < 1e-8


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("prec,coarse", [("f64", -1), ("f32", -1), ("f32", 10)])
def test_threaded_group_vcycle(world, prec, coarse):
    """The partitioned V-cycle through the rank code path (team calls with
    n = 1, as an RCCL rank makes them): one host thread and one stream per
    member, every level's vmult the production dist_vmult schedule with the
    fused relaxation (csrc/dist.hip GroupTransport: device copies gated by
    the peers' events), the redundant direct coarse solve's all-reduce
    through the same transport; against the single-domain V-cycle (same
    tolerances as the lockstep group)."""
    import torch
    import glsamd
    import glsdist
    meshes, cm, params, w, u, hist = _hierarchy(1)
    ref, _ = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision=prec,
                              coarse_n_iterations=coarse)
    g = glsdist.NativeGroupMultigrid(meshes, cm, world, precision=prec,
                                     coarse_n_iterations=coarse)
    g.setup(params, u, hist, w)
    b = gi.rnd(11, meshes[-1].n_dofs)
    bs = g.scatter(b)
    xs = [torch.zeros_like(x) for x in bs]
    g.vcycle_threaded(xs, bs, reps=2)
    src = torch.from_numpy(b).cuda()
    dst = torch.zeros_like(src)
    ref.vcycle(dst, src)
    torch.cuda.synchronize()
    err = rel_err(g.gather(xs).cpu().numpy(), dst.cpu().numpy())
    print(f"threaded world {world} {prec} coarse {coarse}: partitioned vs single-domain "
          f"V-cycle {err:.2e}")
    assert err < (1e-10 if prec == "f64" else 1e-5)


@pytest.mark.parametrize("world", [2, 4])
def test_threaded_group_gmres(world):
    """GMRES over the rank code path (n = 1 per thread): the CGS2 partials
    all-reduced through the in-process transport; against the single-domain
    solve (iterations +-1, solution 1e-8)."""
    import torch
    import glsamd
    import glsdist
    meshes, cm, params, w, u, hist = _hierarchy(1)
    mg, _ = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f64",
                             coarse_n_iterations=-1)
    A = glsamd.NavierStokesOperator(meshes[-1], cm[-1], "f64")
    A.set_parameters(**params)
    A.set_linearization_point(u)
    A.set_previous_solution(hist, w)
    b = gi.rnd(12, meshes[-1].n_dofs)
    src = torch.from_numpy(b).cuda()
    x_ref = torch.zeros_like(src)
    solver = glsamd.LinearSolverGMRES(A, mg, relative_tolerance=1e-8, absolute_tolerance=0.0)
    solver.solve(x_ref, src)
    it_ref = solver.last["n_iterations"]
    g = glsdist.NativeGroupMultigrid(meshes, cm, world, precision="f64", coarse_n_iterations=-1)
    g.setup(params, u, hist, w)
    bs = g.scatter(b)
    xs = [torch.zeros_like(x) for x in bs]
    res = g.gmres_threaded(xs, bs, relative_tolerance=1e-8, absolute_tolerance=0.0)
    torch.cuda.synchronize()
    err = rel_err(g.gather(xs).cpu().numpy(), x_ref.cpu().numpy())
    its = [r["n_iterations"] for r in res]
    print(f"threaded world {world}: GMRES {its} vs {it_ref} iterations, x rel diff {err:.2e}")
    assert all(r["converged"] for r in res) and len(set(its)) == 1
    assert abs(its[0] - it_ref) <= 1
    assert err < 1e-8


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("prec,coarse,n_ref,k", [("f64", 10, 2, 1), ("f32", 10, 2, 1),
                                                 ("f32", -1, 2, 1), ("f64", -1, 1, 1)])
def test_native_group_vcycle_agglomerated(world, prec, coarse, n_ref, k):
    """Level agglomeration (glsDistMGDesc n_redundant_levels, VERDICT r5
    item 4 (ii)): levels 0 .. k-1 plus a copy of level k run single-domain on
    every rank (one all-reduce of level k's right-hand side instead of their
    halo exchanges), levels k .. partitioned; the same V-cycle as the
    single-domain hierarchy (tolerances of the partitioned tests), through
    the lockstep team call and through the rank code path (one thread and
    stream per member)."""
    import torch
    import glsamd
    import glsdist
    meshes, cm, params, w, u, hist = _hierarchy(n_ref)
    ref, _ = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision=prec,
                              coarse_n_iterations=coarse)
    g = glsdist.NativeGroupMultigrid(meshes, cm, world, precision=prec,
                                     coarse_n_iterations=coarse, redundant_levels=k)
    g.setup(params, u, hist, w)
    for l in range(k + 1, len(meshes)):
        wd, lam = g.mg[0].relaxation(l - k)
        wr, lr = ref.relaxation(l)
        assert abs(wd - wr) <= 1e-6 * abs(wr), (l, wd, wr)
    b = gi.rnd(11, meshes[-1].n_dofs)
    src = torch.from_numpy(b).cuda()
    dst = torch.zeros_like(src)
    ref.vcycle(dst, src)
    bs = g.scatter(b)
    xs = [torch.zeros_like(x) for x in bs]
    g.vcycle(xs, bs)
    xt = [torch.zeros_like(x) for x in bs]
    g.vcycle_threaded(xt, bs, reps=2)
    torch.cuda.synchronize()
    tol = 1e-10 if prec == "f64" else 1e-5
    for name, x in (("lockstep", xs), ("threaded", xt)):
        err = rel_err(g.gather(x).cpu().numpy(), dst.cpu().numpy())
        print(f"world {world} {prec} coarse {coarse} levels {n_ref + 1}, {k} agglomerated, {name}:"
              f" vs single-domain V-cycle {err:.2e}")
        assert err < tol


@pytest.mark.parametrize("world", [2, 4])
def test_native_group_gmres_agglomerated(world):
    """GMRES preconditioned by the agglomerated partitioned multigrid (r0, r1
    single-domain on every rank, r2 partitioned; FP64 levels, direct coarse
    solve) against the single-domain solve: iterations +-1, solution 1e-8."""
    import torch
    import glsamd
    import glsdist
    meshes, cm, params, w, u, hist = _hierarchy(2)
    mg, _ = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                             coarse_n_iterations=10)
    A = glsamd.NavierStokesOperator(meshes[-1], cm[-1], "f64")
    A.set_parameters(**params)
    A.set_linearization_point(u)
    A.set_previous_solution(hist, w)
    b = gi.rnd(12, meshes[-1].n_dofs)
    src = torch.from_numpy(b).cuda()
    x_ref = torch.zeros_like(src)
    solver = glsamd.LinearSolverGMRES(A, mg, relative_tolerance=1e-8, absolute_tolerance=0.0)
    solver.solve(x_ref, src)
    it_ref = solver.last["n_iterations"]
    g = glsdist.NativeGroupMultigrid(meshes, cm, world, precision="f32", coarse_n_iterations=10,
                                     redundant_levels=1)
    g.setup(params, u, hist, w)
    bs = g.scatter(b)
    xs = [torch.zeros_like(x) for x in bs]
    res = g.gmres(xs, bs, relative_tolerance=1e-8, absolute_tolerance=0.0)
    torch.cuda.synchronize()
    err = rel_err(g.gather(xs).cpu().numpy(), x_ref.cpu().numpy())
    print(f"world {world} agglomerated: GMRES {res['n_iterations']} vs {it_ref} iterations, "
          f"x rel diff {err:.2e}")
    assert res["converged"] and abs(res["n_iterations"] - it_ref) <= 1
    assert err < 1e-6
