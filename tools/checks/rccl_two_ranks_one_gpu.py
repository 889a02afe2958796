import os, torch, torch.distributed as dist
r = int(os.environ["RANK"]); torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((1 << 20,), r + 1, dtype=torch.uint8, device="cuda")
out = [torch.empty_like(x) for _ in range(2)] if r == 0 else None
dist.gather(x, out, dst=0)
torch.cuda.synchronize()
if r == 0: print("gather ok", [int(o[0]) for o in out])
dist.destroy_process_group()
