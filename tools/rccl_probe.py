"""RCCL smoke probe: one process group of WORLD_SIZE ranks (default: 1 rank
on cuda:0, or the ranks bench.py --gpus N would start), each collective the
sharded path uses, one line printed per step (so a hang names its step).
  python tools/rccl_probe.py            # one rank
  torchrun-less: RANK / WORLD_SIZE / MASTER_* from the environment"""
import os
import socket
import sys
import time


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    t0 = time.time()

    def say(msg):
        print(f"[rank {rank} {time.time() - t0:7.2f}s] {msg}", flush=True)
    eager = "--lazy" not in sys.argv
    say(f"init nccl world {world} ({'eager, device_id' if eager else 'lazy'})")
    if eager:
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("nccl")
    say("init done")
    if "--stream" in sys.argv:  # bench.py's setup: a non-default current stream
        s = torch.cuda.Stream(dev)
        torch.cuda.set_stream(s)
        say("side stream set")
    x = torch.ones(4, device=dev)
    dist.all_reduce(x)
    torch.cuda.synchronize()
    say(f"all_reduce {x.tolist()}")
    g = torch.empty(4 * world, device=dev)
    dist.all_gather_into_tensor(g, x)
    torch.cuda.synchronize()
    say("all_gather_into_tensor")
    c = torch.arange(world, dtype=torch.int64, device=dev)
    r = torch.empty_like(c)
    dist.all_to_all_single(r, c)
    torch.cuda.synchronize()
    say(f"all_to_all_single counts {r.tolist()}")
    rows = torch.arange(3 * 10 * world, dtype=torch.int32, device=dev).view(-1, 3)
    out = torch.empty_like(rows)
    dist.all_to_all_single(out, rows, output_split_sizes=[10] * world,
                           input_split_sizes=[10] * world)
    torch.cuda.synchronize()
    say("all_to_all_single rows [n, 3] with split sizes")
    # the sharded step's empty exchanges (a shard with no halo rows to send
    # or receive: every split zero, as at one rank)
    e_in = torch.empty((0, 3), dtype=torch.int32, device=dev)
    e_out = torch.empty((0, 3), dtype=torch.int32, device=dev)
    say("all_to_all_single of empty tensors, zero splits ...")
    dist.all_to_all_single(e_out, e_in, output_split_sizes=[0] * world,
                           input_split_sizes=[0] * world)
    torch.cuda.synchronize()
    say("all_to_all_single of empty tensors, zero splits")
    big = next((int(a.split("=")[1]) for a in sys.argv if a.startswith("--big=")), 0)
    for it in range(4 if big else 0):
        # a large [rows, 3] exchange (one rank: the identity), checked on the
        # current stream right after the call, then after a device-wide sync
        src = torch.randint(0, 1 << 30, (big, 3), dtype=torch.int32, device=dev)
        dst = torch.empty_like(src)
        dist.all_to_all_single(dst, src, output_split_sizes=[big // world] * world,
                               input_split_sizes=[big // world] * world)
        ordered = int((dst != src).any(dim=1).sum())
        torch.cuda.synchronize()
        after = int((dst != src).any(dim=1).sum())
        say(f"big all_to_all [{big}, 3] #{it}: rows differing, stream-ordered {ordered}, "
            f"after device sync {after}")
    dist.barrier()
    say("barrier")
    dist.destroy_process_group()
    say("done")


if __name__ == "__main__":
    main()
