"""Per-utterance data parallelism over one node.

The reference is single-process, batch 1 (infer.py). Utterances are independent, so each rank
(one process per GPU, torch.distributed with the nccl backend = RCCL over xGMI) converts its own
shard with no data-path collective; the only exchange is the final gather of every rank's output
waveforms to rank 0. Sampler noise is keyed by the global utterance id, so outputs are identical
for any world size.
"""
import os

import torch
import torch.distributed as torchdist


def shard(n_items, rank, world):
    """Contiguous shard [start, stop) of n_items for `rank` (the first n % world ranks get one more)."""
    q, r = divmod(n_items, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


class DistContext:
    def __init__(self, rank=0, world=1, local_rank=0, backend=None):
        self.rank, self.world, self.local_rank, self.backend = rank, world, local_rank, backend

    @classmethod
    def from_env(cls, backend=None):
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if world > 1 and not torchdist.is_initialized():
            backend = backend or ("nccl" if torch.cuda.is_available() else "gloo")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if backend == "nccl":
                torch.cuda.set_device(local)
                torchdist.init_process_group(backend, device_id=torch.device("cuda", local))
            else:
                torchdist.init_process_group(backend)
        return cls(rank, world, local, backend)

    def barrier(self):
        if self.world > 1:
            torchdist.barrier()

    def max_over_ranks(self, value):
        if self.world == 1:
            return value
        dev = "cuda" if self.backend == "nccl" else "cpu"
        t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
        torchdist.all_reduce(t, op=torchdist.ReduceOp.MAX)
        return float(t.item())

    def gather_waveforms(self, wav):
        """Gather every rank's [B_r, S] waveforms to rank 0 -> [sum B_r, S] on rank 0, None elsewhere.
        Shards of unequal size are padded to the largest B (lengths exchanged first)."""
        if self.world == 1:
            return wav
        n = torch.tensor([wav.shape[0]], dtype=torch.int64, device=wav.device)
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        torchdist.all_gather(sizes, n)
        sizes = [int(s.item()) for s in sizes]
        bmax = max(sizes)
        if wav.shape[0] < bmax:
            pad = torch.zeros(bmax - wav.shape[0], *wav.shape[1:], dtype=wav.dtype, device=wav.device)
            wav = torch.cat([wav, pad])
        bufs = [torch.empty_like(wav) for _ in range(self.world)] if self.rank == 0 else None
        torchdist.gather(wav.contiguous(), gather_list=bufs, dst=0)
        if self.rank != 0:
            return None
        return torch.cat([b[:s] for b, s in zip(bufs, sizes)])

    def close(self):
        if self.world > 1 and torchdist.is_initialized():
            torchdist.destroy_process_group()
