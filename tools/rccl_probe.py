"""Probe: can two RCCL ranks share one GPU (the one-GPU box)?  Two processes, torch.distributed 'nccl'
on cuda:0, one all_gather.  Prints 'rccl two ranks on one GPU: ok' or the error; exits 0 either way."""

import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=2, device_id=torch.device("cuda", 0))
        x = torch.full((4,), float(rank), device="cuda:0")
        out = torch.empty(8, device="cuda:0")
        dist.all_gather_into_tensor(out, x)
        torch.cuda.synchronize()
        q.put((rank, out.cpu().tolist()))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, f"error: {type(e).__name__}: {e}"))


def main():
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = []
    for _ in ps:
        try:
            res.append(q.get(timeout=60))
        except Exception as e:  # noqa: BLE001
            res.append(("?", f"timeout: {e}"))
    for p in ps:
        p.join(timeout=10)
        if p.is_alive():
            p.kill()
    ok = all(isinstance(v, list) and v == [0.0] * 4 + [1.0] * 4 for _, v in res)
    print("rccl two ranks on one GPU:", "ok" if ok else res, flush=True)
    sys.exit(0)


if __name__ == "__main__":
    main()
