"""One-rank RCCL smoke on the GPU box: the nccl init_process_group(device_id=...) call and the
barrier / all_reduce(MAX) that bench.py's multi-rank timing uses (fmpnp.shard.timed_steps)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
dist.init_process_group("nccl", device_id=torch.device("cuda", 0), rank=0, world_size=1)
from fmpnp import shard  # noqa: E402

x = torch.full((1,), 3.5, device="cuda:0")
dist.all_reduce(x, op=dist.ReduceOp.MAX)
dist.barrier()
el = shard.timed_steps(lambda k: torch.cuda._sleep(1000), 5, device=torch.device("cuda", 0))
print("rccl ok:", dist.get_backend(), float(x), f"timed_steps {el:.6f} s")
dist.destroy_process_group()
