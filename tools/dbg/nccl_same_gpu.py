"""Probe: can two ranks share one GPU under backend "nccl" (RCCL) on this pool?  If so,
bench.py's N > 1 legs (ScatterIngest / RecordGather over RCCL) can be rehearsed on a
one-GPU box: python -m torch.distributed.run --nproc-per-node 2 tools/dbg/nccl_same_gpu.py"""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.full((4,), float(rank), device="cuda")
if rank == 0:
    dist.recv(t, src=1)
else:
    dist.send(t, dst=0)
torch.cuda.synchronize()
g = dist.new_group([0, 1])
u = torch.full((2,), 10.0 + rank, device="cuda")
w = dist.batch_isend_irecv([dist.P2POp(dist.irecv if rank == 0 else dist.isend, u, 1 - rank, group=g)])
for x in w:
    x.wait()
torch.cuda.synchronize()
print("rank", rank, "ok", t.tolist(), u.tolist(), flush=True)
dist.barrier()
dist.destroy_process_group()
