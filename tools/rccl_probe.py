"""Diagnostic: a one-rank RCCL communicator bootstrapped over loopback (NCCL_SOCKET_IFNAME=lo,
the single-node default of dist.HostGroup) initializes and all-reduces on this box."""
import os, torch, torch.distributed as dist
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", RANK="0", WORLD_SIZE="1", NCCL_SOCKET_IFNAME="lo")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
t = torch.ones(1024, device="cuda:0")
dist.all_reduce(t)
torch.cuda.synchronize()
print("rccl over lo ok", float(t.sum()))
dist.destroy_process_group()
