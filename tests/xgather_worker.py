"""One rank of the multi-process one-shot exchange test (tests/test_gpu_exchange.py): started
as a child process (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the environment) on the
box's one GPU, joins a gloo process group (the handle exchange and the digest all-gathers),
maps every rank's receive region through HIP IPC (ragen_amd.exchange.ArenaExchange) and runs
EPOCHS exchanges of an nbytes arena whose content depends on (rank, epoch), one fused launch
each.  After every exchange it checks the gathered slot against every rank's expected bytes
(each rank can regenerate every other rank's arena) and, every DIGEST_EVERY epochs, against
the digests the owners all-gathered (bench.arena_digests).  Writes <out>/rank<r>.json."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ragen_amd.exchange import ArenaExchange  # noqa: E402


def arena(rank, epoch, nbytes, device, base):
    """The rank's arena at an epoch: its base bytes xor a (rank, epoch) byte pattern."""
    k = (rank * 131 + epoch * 29) & 255
    return base[rank] ^ torch.tensor(k, dtype=torch.uint8, device=device)


def main():
    out, nbytes, epochs = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    digest_every = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    dist.init_process_group("gloo")
    W, r = dist.get_world_size(), dist.get_rank()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from bench import arena_digests
    g = torch.Generator(device="cpu").manual_seed(1234)
    base = [torch.randint(0, 256, (nbytes,), dtype=torch.uint8, generator=g).to(dev) for _ in range(W)]
    ex = ArenaExchange(nbytes, dev, timeout_us=5_000_000)
    bad, digest_checks = [], 0
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    t0 = time.perf_counter()
    for e in range(1, epochs + 1):
        src.copy_(arena(r, e, nbytes, dev, base))
        ex.run(src)
        got = ex.slot()
        want = torch.stack([arena(q, e, nbytes, dev, base) for q in range(W)])
        if not torch.equal(got, want):
            bad.append(e)
        if e % digest_every == 0:  # the owners' digests, all-gathered (gloo: host tensors)
            mine = arena_digests(src.view(1, -1)).cpu()
            every = [torch.zeros_like(mine) for _ in range(W)]
            dist.all_gather(every, mine)
            have = arena_digests(got.contiguous()).cpu().view(W, -1)
            if not all(torch.equal(have[q].view(-1), every[q].view(-1)) for q in range(W)):
                bad.append(-e)
            digest_checks += 1
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    err = ex.error()
    dist.barrier()  # nobody unmaps a region a peer may still store into
    ex.close()
    with open(os.path.join(out, f"rank{r}.json"), "w") as f:
        json.dump({"rank": r, "world": W, "epochs": ex.epoch, "bad": bad, "err": err,
                   "digest_checks": digest_checks, "seconds": dt}, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
