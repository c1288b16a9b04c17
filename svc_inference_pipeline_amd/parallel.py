"""Per-utterance data parallelism over one node.

The reference is single-process, batch 1 (infer.py). Utterances are independent, so each rank
(one process per GPU, torch.distributed with the nccl backend = RCCL over xGMI) converts its own
shard with no data-path collective; the only exchange is the final gather of every rank's output
waveforms to rank 0. Sampler noise is keyed by the global utterance id, so outputs are identical
for any world size.
"""
import datetime
import os

import torch
import torch.distributed as torchdist


def shard(n_items, rank, world):
    """Contiguous shard [start, stop) of n_items for `rank` (the first n % world ranks get one more)."""
    q, r = divmod(n_items, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


DEFAULT_TIMEOUT_S = 600.0  # rendezvous and every collective; SVC_DIST_TIMEOUT_S overrides


class DistContext:
    def __init__(self, rank=0, world=1, local_rank=0, backend=None):
        self.rank, self.world, self.local_rank, self.backend = rank, world, local_rank, backend

    @classmethod
    def from_env(cls, backend=None, timeout_s=None):
        """One rank of a torch.distributed.run / bench.spawn_ranks launch (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_*).
        Collectives time out after `timeout_s` (default SVC_DIST_TIMEOUT_S or 600 s): a rank whose peer hangs
        raises instead of waiting forever, so the launcher sees it exit and can end the job."""
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if world > 1 and not torchdist.is_initialized():
            backend = backend or ("nccl" if torch.cuda.is_available() else "gloo")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if timeout_s is None:
                timeout_s = float(os.environ.get("SVC_DIST_TIMEOUT_S", DEFAULT_TIMEOUT_S))
            timeout = datetime.timedelta(seconds=timeout_s)
            if backend == "nccl":
                torch.cuda.set_device(local)
                torchdist.init_process_group(backend, timeout=timeout, device_id=torch.device("cuda", local))
            else:
                torchdist.init_process_group(backend, timeout=timeout)
        if torchdist.is_initialized():  # the process group's own view (what rank 0 reports)
            world, rank = torchdist.get_world_size(), torchdist.get_rank()
            backend = str(torchdist.get_backend())
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

    def all_gather_floats(self, values):
        """Every rank's list of floats (same length on every rank) -> [world][len] on every rank."""
        if self.world == 1:
            return [list(map(float, values))]
        dev = "cuda" if self.backend == "nccl" else "cpu"
        t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=dev)
        out = [torch.empty_like(t) for _ in range(self.world)]
        torchdist.all_gather(out, t)
        return [o.cpu().tolist() for o in out]

    def gather_waveforms(self, wav, lengths=None, return_lengths=False):
        """Gather every rank's [B_r, S_r] waveforms to rank 0 -> [sum B_r, max S_r] on rank 0, None elsewhere.

        The (B_r, S_r) shapes are all-gathered first (one int64 pair per rank); each shard is zero-padded to the
        largest B and S, so ranks may hold different numbers of utterances and different clip lengths.
        `lengths` (int [B_r], default S_r for every row) are the per-utterance valid sample counts; with
        `return_lengths` rank 0 also gets them for the whole gathered batch (int64 [sum B_r], None elsewhere).
        A 1-D wav is one utterance ([1, S_r])."""
        if wav.dim() == 1:
            wav = wav.reshape(1, -1)
        if wav.dim() != 2:
            raise ValueError(f"gather_waveforms: wav must be [B, S] or [S], got {tuple(wav.shape)}")
        if lengths is None:
            lengths = torch.full((wav.shape[0],), wav.shape[1], dtype=torch.int64)
        lengths = torch.as_tensor(lengths, dtype=torch.int64)
        if self.world == 1:
            return (wav, lengths) if return_lengths else wav
        dev = wav.device
        shape = torch.tensor([wav.shape[0], wav.shape[1]], dtype=torch.int64, device=dev)
        shapes = [torch.zeros_like(shape) for _ in range(self.world)]
        torchdist.all_gather(shapes, shape)
        shapes = [(int(s[0].item()), int(s[1].item())) for s in shapes]
        bmax = max(b for b, _ in shapes)
        smax = max(s for _, s in shapes)
        buf = torch.zeros(bmax, smax, dtype=wav.dtype, device=dev)
        if wav.numel():
            buf[:wav.shape[0], :wav.shape[1]] = wav
        lbuf = torch.zeros(bmax, dtype=torch.int64, device=dev)
        lbuf[:lengths.numel()] = lengths.to(dev)
        bufs = [torch.empty_like(buf) for _ in range(self.world)] if self.rank == 0 else None
        lbufs = [torch.empty_like(lbuf) for _ in range(self.world)] if self.rank == 0 else None
        torchdist.gather(buf, gather_list=bufs, dst=0)
        torchdist.gather(lbuf, gather_list=lbufs, dst=0)
        if self.rank != 0:
            return (None, None) if return_lengths else None
        out = torch.cat([b[:n] for b, (n, _) in zip(bufs, shapes)])
        if return_lengths:
            return out, torch.cat([l[:n] for l, (n, _) in zip(lbufs, shapes)]).cpu()
        return out

    def close(self):
        if self.world > 1 and torchdist.is_initialized():
            torchdist.destroy_process_group()
