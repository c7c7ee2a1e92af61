"""Does an RCCL all-reduce capture into a HIP graph? (GPU box, one rank)

A 1-rank nccl (= RCCL) process group; dist.all_reduce of a bucket issued (a) on a side stream
forked inside torch.cuda.graph capture and joined back, (b) on the capture stream itself.  Each
graph is replayed a few times with the bucket refilled between replays; prints whether capture
and replay succeed and whether the replayed sum (the identity for one rank, x2 for a bucket added
to itself first) is right.  If it does, the trainer's split captures (one graph per bucket hook,
the all-reduce issued between replays) could become one graph with the collective as a node."""
import os
import socket
import sys

import torch
import torch.distributed as dist


def main():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    x = torch.zeros(25 << 18, device=dev)  # 25 MiB of fp32, one DDP bucket
    dist.all_reduce(x)  # communicator warm-up outside any capture
    torch.cuda.synchronize()
    for mode in ("side", "same"):
        try:
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream(device=dev)
            with torch.cuda.graph(g):
                x.mul_(2.0)
                if mode == "side":
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(side):
                        dist.all_reduce(x)
                    torch.cuda.current_stream().wait_stream(side)
                else:
                    dist.all_reduce(x)
                x.add_(1.0)
            ok = True
            for i in range(3):
                x.fill_(float(i))
                g.replay()
                torch.cuda.synchronize()
                ok &= bool(torch.all(x == 2.0 * i + 1.0))
            print(f"{mode}: capture ok, replay {'correct' if ok else 'WRONG'}", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"{mode}: FAILED {type(e).__name__}: {str(e)[:300]}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
