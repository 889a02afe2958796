"""One-rank RCCL check of the per-step label gather (the multi-GPU bench path):
python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 tools/nccl_gather_check.py"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vad_amd.dist import LabelGather, gather_labels  # noqa: E402

dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
g = LabelGather(1000, dev)
x = (torch.arange(1000, device=dev) % 3).to(torch.uint8)
out = g(x)
torch.cuda.synchronize()
assert g._use_gather, "nccl gather refused"
assert torch.equal(out[0], x)
out2 = gather_labels(x[:7])
assert torch.equal(out2[0], x[:7])
print("nccl gather ok, point-to-point:", g._use_gather)
dist.destroy_process_group()
