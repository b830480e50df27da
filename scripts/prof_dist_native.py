"""Native partitioned multigrid + GMRES (gls_dist_mg_vcycle,
gls_dist_gmres_solve) at world 1 over RCCL: 3 GMRES(28) solves of 28
iterations each on the Re3900 r0..r2 hierarchy, FP32 levels, coarse 10
relaxation sweeps (for rocprofv3 --kernel-trace --stats; wall time printed)."""
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

with socket.socket() as sk:
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
import glsamd  # noqa: E402
import glsdist  # noqa: E402
import glsinputs as gi  # noqa: E402
import glsmesh as gm  # noqa: E402

d = gm.read_deck(os.path.join(gm.DECK_DIR, "input_hoffmann_3D_Re3900.json"))
params, w = d.operator_parameters(2.5e-4)
meshes = [d.mesh(r) for r in range(3)]
vel, p, slip = d.boundary_descriptor()
cm = [m.constraint_mask(vel, p, slip) for m in meshes]
u = gi.linearization_point(meshes[-1].n_nodes, 3, d.u_max)
hist = gi.history(u, params["order"])
dmg = glsdist.DistributedMultigrid(meshes, cm, "f32", dist, 0, 1, coarse_n_iterations=10)
A = dmg.fine_operator("f64")
A.setup(params, u, hist, w)
mg = dmg.native(params, u, hist, w)
b = A.scatter_global(gi.src_vector(meshes[-1].n_dofs))
x = A.new_vector()


def solve():
    try:
        glsamd.dist_gmres_solve([A.native], [mg], [x], [b], n_max_iterations=28,
                                relative_tolerance=0.0, absolute_tolerance=0.0)
    except glsamd.GlsError:
        pass


solve()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    solve()
torch.cuda.synchronize()
print(f"native dist GMRES iteration {(time.perf_counter() - t0) / 84 * 1e3:.3f} ms")
dist.destroy_process_group()
