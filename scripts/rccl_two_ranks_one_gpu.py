#!/usr/bin/env python3
"""RCCL with peers on ONE GPU: two ranks (torch.distributed.run
--nproc-per-node 2) both on device 0, the native partitioned vmult
(gls_dist_vmult over RcclTransport: ghost import / export between the two
ranks) against the single-domain vmult of the same inputs.  RCCL may refuse
two ranks on one device; the script then reports that and exits 2."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))


def main():
    import torch
    import torch.distributed as dist
    import glsamd
    import glsdist
    import glsinputs as gi
    import glsmesh as gm
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    try:
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        t = torch.ones(1, device="cuda")
        dist.all_reduce(t)
        torch.cuda.synchronize()
    except Exception as e:  # RCCL's verdict on two ranks per device
        print(f"rank {rank}: RCCL refused two ranks on one GPU: {e}", flush=True)
        sys.exit(2)
    d = gm.read_deck(os.path.join(gm.DECK_DIR, "input_hoffmann_3D_Re3900.json"))
    m = d.mesh(int(os.environ.get("NREF", "1")))
    cm = m.constraint_mask(*d.boundary_descriptor())
    prm, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(m.n_nodes, m.dim, d.u_max)
    hist = gi.history(u, prm["order"])
    op = glsdist.DistributedOperator(m, cm, "f64", dist, rank, world)
    assert op.native is not None
    op.setup(prm, u, hist, w)
    src_g = torch.from_numpy(gi.src_vector(m.n_dofs)).cuda()
    src = op.scatter_global(src_g)
    dst = op.new_vector()
    for _ in range(3):
        op.vmult(dst, src)
    torch.cuda.synchronize()
    g = op.gather_global(dst)
    ref_op = glsamd.NavierStokesOperator(m, cm, "f64")
    ref_op.set_parameters(**prm)
    ref_op.set_linearization_point(u)
    if prm["order"] > 0:
        ref_op.set_previous_solution(hist, w)
    ref = ref_op.initialize_dof_vector()
    ref_op.vmult(ref, src_g)
    torch.cuda.synchronize()
    err = float(torch.linalg.norm(g - ref) / torch.linalg.norm(ref))
    peers = len(op.r.part.recv_nodes) if hasattr(op.r.part, "recv_nodes") else -1
    print(f"rank {rank}/{world}: peers {peers}, owned dofs {op.r.n_owned_dofs}, "
          f"partitioned vs single-domain vmult rel l2 {err:.2e}", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if err < 1e-12 else 1)


if __name__ == "__main__":
    main()
