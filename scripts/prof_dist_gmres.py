"""Host profile (cProfile) of the partitioned multigrid + GMRES iteration at
world 1 (GLS_BENCH_DIST rehearsal): where the host-driven orchestration
spends its time."""
import cProfile
import os
import pstats
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

with socket.socket() as sk:
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
import bench  # noqa: E402
import glsmesh as gm  # noqa: E402

d = gm.read_deck(os.path.join(gm.DECK_DIR, bench.DECK))
params, weights = d.operator_parameters(2.5e-4)
bench.dist_gmres_companion(d, params, weights, 2, dist, 0, 1, reps=3)
pr = cProfile.Profile()
pr.enable()
t0 = time.perf_counter()
out = bench.dist_gmres_companion(d, params, weights, 2, dist, 0, 1, reps=10)
pr.disable()
print(out, time.perf_counter() - t0)
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
dist.destroy_process_group()
