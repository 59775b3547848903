"""One rank of the sharded GPU batch (run under torch.distributed.run by
tests/test_gpu_parity.py::test_ranks_shard_a_batch_on_the_gpu, never
collected by pytest): rank r CRCs its byte-balanced slice of a Zipf batch
through the HIP path (bmqcrc_crc32c_batch, device-resident, payload generated
in HBM), checks every CRC of the slice against the oracle, and rank 0
stitches the gathered slices and checks them against the whole batch.  The
device is rank % device_count: one GPU on a one-GPU box, distinct GPUs on a
node.  gloo carries only the results for the assertion (the product has no
data-path collective).  Exit status 0 = bit-exact."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    import oracle
    from blazingmq_amd import Crc32c, fill_synthetic
    from blazingmq_amd.shard import rank_slice

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", rank % ndev)
    torch.cuda.set_device(dev)
    rng = np.random.default_rng(77)
    r = np.arange(1, 16385, dtype=np.float64)
    p = r ** -1.5
    p /= p.sum()
    lens = (64 * rng.choice(16384, size=20000, p=p) + rng.integers(0, 64, size=20000)).astype(
        np.uint32)
    lo, hi = rank_slice(lens, rank, world)
    begin = int(lens[:lo].sum(dtype=np.uint64)) & ~7  # fill streams start 8-byte aligned
    pad = int(lens[:lo].sum(dtype=np.uint64)) - begin
    mine = lens[lo:hi]
    offs = (pad + np.concatenate([[0], np.cumsum(mine, dtype=np.uint64)[:-1]])).astype(np.int64)
    nbytes = pad + int(mine.sum(dtype=np.uint64))
    arena = torch.empty(max(nbytes, 8) + 8, dtype=torch.uint8, device=dev)
    fill_synthetic(arena, 9, begin=begin)
    seeds = rng.integers(0, 2**32, size=lens.size, dtype=np.uint64).astype(np.uint32)
    got = Crc32c.calculate_batch(
        arena, torch.from_numpy(offs).to(dev), torch.from_numpy(mine.view(np.int32)).to(dev),
        torch.from_numpy(seeds[lo:hi].view(np.int32)).to(dev)).cpu().numpy().view(np.uint32)
    host = oracle.fill_payload(begin, nbytes, 9)
    exp = oracle.batch(host, offs.astype(np.uint64), mine, seeds=seeds[lo:hi], nthreads=4)
    ok_slice = bool(np.array_equal(got, exp))
    gathered = [None] * world
    dist.all_gather_object(gathered, (lo, hi, got.tolist(), ok_slice, str(dev)))
    status = 0
    if rank == 0:
        full_host = oracle.fill_payload(0, int(lens.sum(dtype=np.uint64)), 9)
        full_offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
        full = oracle.batch(full_host, full_offs, lens, seeds=seeds, nthreads=4).tolist()
        stitched = []
        for lo_r, hi_r, res, _, _ in sorted(gathered):
            stitched += res
        ok = stitched == full and all(g[3] for g in gathered)
        print("ranks=%d devices=%s slices=%s bit_exact=%s" % (
            world, [g[4] for g in gathered], [(g[0], g[1]) for g in gathered], ok), flush=True)
        status = 0 if ok else 1
    dist.barrier()
    dist.destroy_process_group()
    return status


if __name__ == "__main__":
    sys.exit(main())
