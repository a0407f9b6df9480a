"""GPU box probe: can two RCCL ranks share the one GPU of the box?  Two processes, backend nccl, both on
cuda:0, one all_reduce + barrier.  Prints RCCL_OK <value> from rank 0 or the error."""
import os
import sys
import torch
import torch.distributed as dist


def main():
    dist.init_process_group("nccl")
    torch.cuda.set_device(0)
    t = torch.full((1024,), float(dist.get_rank() + 1), device="cuda:0")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    dist.barrier()
    if dist.get_rank() == 0:
        print("RCCL_OK", float(t[0]), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
