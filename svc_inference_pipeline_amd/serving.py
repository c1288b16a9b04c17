"""Streaming request front end over the ragged-batch pipeline.

The reference converts one clip per call (infer.py:44-90, B = 1 throughout). A service receives clips one at a time
and of any length; SVCServer turns that stream into ragged GPU batches:

    server = SVCServer(SVCPipeline(engine), max_batch=32, max_wait_s=0.02)
    fut = server.submit(wav24, wav16, singer_id)       # returns at once (concurrent.futures.Future)
    wav = fut.result()                                 # f32 [T * hop] on the GPU
    server.close()

A worker thread takes the oldest pending request, adds the pending requests whose length is within `length_ratio` of
it (so padding stays bounded: the kernels skip the padded tail, but its rows still occupy the batch) up to
`max_batch`, waits at most `max_wait_s` for a batch to fill, and runs SVCPipeline.convert_ragged on it. Each request
carries an utterance id (given, or a running counter) that keys its device noise, so its waveform is bit-identical to
converting that clip alone with the same id, whatever it was batched with (tests/test_gpu_ragged.py).

Streams: submit() records an event on the caller's current stream, and the worker's stream waits for it before it
reads the request's tensors, so inputs produced by kernels still in flight on the caller's stream are safe to
submit. A result is a view into the batch's output, recorded for use on the submitting stream (record_stream), and
the future resolves once it is complete. The engine's lock (SVCEngine.lock) serialises the worker's conversions with
any direct use of the same engine.
"""
import collections
import itertools
import threading
import time
from concurrent.futures import Future
from dataclasses import dataclass, field

import torch

from .pipeline import SVCPipeline
from .runtime import mel_frames


@dataclass
class _Request:
    wav24: torch.Tensor
    wav16: torch.Tensor
    singer: int
    utt_id: int
    wav16_float: torch.Tensor = None
    frames: int = 0
    t_submit: float = 0.0
    ready: object = None    # torch.cuda.Event recorded on the submitting stream (None on the CPU)
    stream: object = None   # the submitting stream
    future: Future = field(default_factory=Future)


class SVCServer:
    def __init__(self, pipeline: SVCPipeline, max_batch=32, max_wait_s=0.02, length_ratio=2.0, fast_inference=True,
                 speedup=10, seed=0):
        if max_batch < 1 or max_wait_s < 0 or length_ratio < 1.0:
            raise ValueError("SVCServer: max_batch >= 1, max_wait_s >= 0, length_ratio >= 1")
        self.pipeline = pipeline
        self.max_batch = int(max_batch)
        self.max_wait_s = float(max_wait_s)
        self.length_ratio = float(length_ratio)
        self.kw = dict(fast_inference=fast_inference, speedup=speedup, seed=seed)
        cfg = pipeline.engine.cfg
        self._frames = lambda n: mel_frames(n, cfg.n_fft, cfg.hop_length)
        self._ids = itertools.count()
        self._pending = []
        self._cv = threading.Condition()
        self._closed = False
        self.batches = collections.deque(maxlen=4096)  # utterance ids of the most recent batches (inspection, tests)
        self._device = getattr(pipeline.engine, "device", None)
        self._worker = threading.Thread(target=self._run, name="svc-server", daemon=True)
        self._worker.start()

    def submit(self, wav24, wav16, singer, utt_id=None, wav16_float=None) -> Future:
        """Queue one utterance (device tensors: 24 kHz f32 [N], 16 kHz [N16], optional float 16 kHz for
        ContentVec) -> Future resolving to its waveform f32 [T * hop]."""
        n = int(wav24.shape[-1])
        if n < 1 or int(wav16.shape[-1]) < 1:
            raise ValueError("SVCServer.submit: empty audio")
        req = _Request(wav24=wav24.reshape(-1), wav16=wav16.reshape(-1), singer=int(singer),
                       utt_id=next(self._ids) if utt_id is None else int(utt_id),
                       wav16_float=None if wav16_float is None else wav16_float.reshape(-1),
                       frames=self._frames(n), t_submit=time.monotonic())
        if wav24.is_cuda:
            req.stream = torch.cuda.current_stream(wav24.device)
            req.ready = torch.cuda.Event()
            req.ready.record(req.stream)
        with self._cv:
            if self._closed:
                raise RuntimeError("SVCServer.submit: the server is closed")
            self._pending.append(req)
            self._cv.notify()
        return req.future

    def close(self, wait=True):
        """Stop accepting requests; the worker finishes every queued request first."""
        with self._cv:
            self._closed = True
            self._cv.notify()
        if wait:
            self._worker.join()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ------------------------------------------------------------------ worker
    def _take_batch(self):
        """The oldest request plus the pending ones of compatible length (within length_ratio, same ContentVec input
        form), at most max_batch; called with the lock held."""
        head = self._pending[0]
        lo, hi = head.frames / self.length_ratio, head.frames * self.length_ratio
        batch = [head]
        for r in self._pending[1:]:
            if len(batch) == self.max_batch:
                break
            if lo <= r.frames <= hi and (r.wav16_float is None) == (head.wav16_float is None):
                batch.append(r)
        taken = set(map(id, batch))
        self._pending = [r for r in self._pending if id(r) not in taken]
        return batch

    def _ready(self):
        """A batch may run: it is full, the oldest request has waited max_wait_s, or the server is closing."""
        if not self._pending:
            return False
        if self._closed or len(self._pending) >= self.max_batch:
            return True
        return time.monotonic() - self._pending[0].t_submit >= self.max_wait_s

    def _run(self):
        if self._device is not None and torch.cuda.is_available():
            torch.cuda.set_device(self._device)
        while True:
            with self._cv:
                while not self._ready():
                    if self._closed and not self._pending:
                        return
                    timeout = None
                    if self._pending:
                        timeout = max(0.0, self.max_wait_s - (time.monotonic() - self._pending[0].t_submit))
                    self._cv.wait(timeout)
                batch = self._take_batch()
            self._convert(batch)

    def _convert(self, batch):
        try:
            if torch.cuda.is_available():
                work = torch.cuda.current_stream()
                for r in batch:  # the inputs' producers on the submitting streams
                    if r.ready is not None:
                        work.wait_event(r.ready)
                    for t in (r.wav24, r.wav16, r.wav16_float):
                        if t is not None and t.is_cuda:
                            t.record_stream(work)
            w16f = [r.wav16_float for r in batch] if batch[0].wav16_float is not None else None
            wavs = self.pipeline.convert_ragged([r.wav24 for r in batch], [r.wav16 for r in batch],
                                                [r.singer for r in batch], wavs16_float=w16f,
                                                utt_ids=[r.utt_id for r in batch], **self.kw)
            if torch.cuda.is_available():
                torch.cuda.current_stream().synchronize()
            self.batches.append([r.utt_id for r in batch])
            for r, w in zip(batch, wavs):
                if r.stream is not None and w.is_cuda:
                    w.record_stream(r.stream)  # the batch buffer outlives the consumer's use on its own stream
                r.future.set_result(w)
        except Exception as exc:  # noqa: BLE001 - every waiting caller gets the failure
            for r in batch:
                if not r.future.done():
                    r.future.set_exception(exc)
