"""Throughput benchmark: converted audio seconds per second (RTF^-1), end-to-end, 10 s clips.

BASELINE.json configs[1]: batch = 32 synthetic 10 s clips per GPU, Whisper-medium content + 100-step
DiffSVC (the reference's PLMS path, speedup 10 = 101 denoiser calls) + BigVGAN. One "step" = the
whole hot path over one batch already resident in HBM: mel/energy, Praat-AC F0, pitch shift,
Whisper log-mel + encoder, content map, conditioner, PLMS-100 sampler, de-normalisation, BigVGAN,
fade-out, and (N > 1) the RCCL gather of every rank's waveforms to rank 0.

    python bench.py [--gpus N --steps K --warmup W]

N > 1: either launched by torch.distributed.run (RANK / LOCAL_RANK / WORLD_SIZE set, one process per GPU), or, when
WORLD_SIZE is unset, this process spawns the N ranks itself (spawn_ranks) BEFORE anything touches the GPU and exits
with the worst rank's status. `--dry-run` replaces the engine by an identity "conversion" of the synthetic clips on
the CPU (gloo), so the spawn / sharding / gather path can be tested without a GPU (tests/test_parallel.py).

Weights are seeded random tensors of the reference architectures (no checkpoints offline); inputs
are synthetic harmonic clips. Rank 0 prints one JSON line.
"""
import argparse
import json
import re
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as torchdist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from svc_inference_pipeline_amd import _lib  # noqa: E402
from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd import weights as W  # noqa: E402
from svc_inference_pipeline_amd.parallel import DistContext  # noqa: E402
from svc_inference_pipeline_amd.pipeline import SVCPipeline  # noqa: E402
from svc_inference_pipeline_amd.runtime import SVCEngine  # noqa: E402

PEAK_F16_TFLOPS = 2500.0   # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def synth_inputs(uids, seconds, float16k=False):
    """24 kHz f32 clips and their 16 kHz copies: int16-quantised for Whisper (ffmpeg s16le,
    utils/whisper_extractor/audio.py:41-49), float for ContentVec (librosa, utils/hubert.py:55)."""
    from svc_inference_pipeline_amd.synth import synth_clip, synth_clip_16k_quantised
    w24 = np.stack([synth_clip(int(u), seconds, 24000) for u in uids])
    if float16k:
        w16 = np.stack([synth_clip(int(u), seconds, 16000) for u in uids]).astype(np.float32)
    else:
        w16 = np.stack([synth_clip_16k_quantised(int(u), seconds) for u in uids])
    return w24, w16


def host_cpus():
    """CPUs this process may use: the scheduler affinity mask, capped by a cgroup CPU quota when one is set
    (a GPU box's process sees the whole machine in nproc but gets a share of it). -> (threads, info dict)."""
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    threads = min(affinity, quota) if quota else affinity
    return threads, {"nproc": affinity, "cgroup_quota_cpus": quota, "cpu_model": model,
                     "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


class ClockSampler:
    """The bench GPU's shader (SCLK) and memory (MCLK) clocks, read in-process from sysfs while the timed region runs
    (a thread reading the card's pp_dpm_sclk / pp_dpm_mclk current level and hwmon's measured sclk every `period` s; no
    subprocess), so that a box-speed shift shows next to `value`. Falls back to the amdsmi Python API when the card's
    sysfs files are not readable. Every failure leaves the fields null with the reason."""

    def __init__(self, device, period=0.05):
        import threading
        self.period = period
        self.samples = []  # (t, sclk_dpm, mclk_dpm, sclk_hwmon) in MHz (None where unread)
        self.err = None
        self.src = None
        self._stop = threading.Event()
        self._thread = None
        self._smi = None
        self.files = {}
        try:
            p = torch.cuda.get_device_properties(device)
            pci = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
            root = f"/sys/bus/pci/devices/{pci}"
            self.pci = pci
            for k, f in (("sclk", "pp_dpm_sclk"), ("mclk", "pp_dpm_mclk")):
                if os.access(os.path.join(root, f), os.R_OK):
                    self.files[k] = os.path.join(root, f)
            hw = os.path.join(root, "hwmon")
            if os.path.isdir(hw):
                for h in sorted(os.listdir(hw)):
                    lab = os.path.join(hw, h, "freq1_label")
                    if os.path.exists(lab) and open(lab).read().strip() == "sclk":
                        self.files["sclk_hwmon"] = os.path.join(hw, h, "freq1_input")
            if self.files:
                self.src = f"sysfs {root}"
            else:
                self._smi_init(p)
        except Exception as e:  # noqa: BLE001 (reported, never fatal)
            self.err = f"{type(e).__name__}: {e}"

    def _smi_init(self, props):
        import amdsmi
        amdsmi.amdsmi_init()
        want = props.pci_bus_id
        for h in amdsmi.amdsmi_get_processor_handles():
            bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)
            if int(bdf.split(":")[1], 16) == want:
                self._smi = (amdsmi, h)
                self.src = f"amdsmi {bdf}"
                return
        raise RuntimeError("no amdsmi handle for the bench GPU")

    @staticmethod
    def _dpm_now(path):
        for line in open(path):
            if line.rstrip().endswith("*"):
                return float(re.search(r"(\d+)\s*[Mm]hz", line).group(1))
        return None

    def read(self):
        sc = mc = hw = None
        if self._smi:
            amdsmi, h = self._smi
            sc = float(amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX)["clk"])
            mc = float(amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.MEM)["clk"])
        else:
            if "sclk" in self.files:
                sc = self._dpm_now(self.files["sclk"])
            if "mclk" in self.files:
                mc = self._dpm_now(self.files["mclk"])
            if "sclk_hwmon" in self.files:
                hw = int(open(self.files["sclk_hwmon"]).read()) / 1e6
        return sc, mc, hw

    def _run(self):
        t0 = time.perf_counter()
        while not self._stop.is_set():
            try:
                self.samples.append((time.perf_counter() - t0,) + self.read())
            except Exception as e:  # noqa: BLE001
                self.err = f"{type(e).__name__}: {e}"
                return
            self._stop.wait(self.period)

    def start(self):
        import threading
        if self.src and not self.err:
            self._thread = threading.Thread(target=self._run, daemon=True)
            self._thread.start()

    def stop(self):
        if self._thread:
            self._stop.set()
            self._thread.join()
            try:
                self.samples.append((None,) + self.read())  # the end of the timed region
            except Exception as e:  # noqa: BLE001
                self.err = f"{type(e).__name__}: {e}"

    def summary(self):
        out = {"source": self.src, "error": self.err, "samples": len(self.samples),
               "period_s": self.period}
        for i, k in ((1, "sclk_mhz"), (2, "mclk_mhz"), (3, "sclk_hwmon_mhz")):
            v = [smp[i] for smp in self.samples if smp[i] is not None]
            if v:
                out[k] = {"start": v[0], "end": v[-1], "median": float(np.median(v)), "min": min(v), "max": max(v)}
        return out


def calibrate(device, seconds=1.0):
    """A fixed box-speed probe, timed in this process after the timed region: torch.matmul (hipBLASLt) of two 4096 x
    4096 fp16 matrices of seeded random values, back to back for about `seconds`, and a 1 GiB device copy. The same
    code on every box and in every round, so a shift of `value` that the calibration shifts with is the box, not the
    build. -> {"gemm_us": per GEMM, "gemm_tflops", "copy_gbs": read + write bytes / s}"""
    g = torch.Generator(device=f"cuda:{device}").manual_seed(0)
    a = torch.randn(4096, 4096, device=f"cuda:{device}", dtype=torch.float16, generator=g)
    b = torch.randn(4096, 4096, device=f"cuda:{device}", dtype=torch.float16, generator=g)
    for _ in range(5):
        c = a @ b
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 0.2:  # size the loop
        c = a @ b
        n += 1
        torch.cuda.synchronize()
    reps = max(10, int(n * seconds / 0.2))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    gemm_us = e0.elapsed_time(e1) * 1000.0 / reps
    x = torch.empty(1 << 29, device=f"cuda:{device}", dtype=torch.float16)
    y = torch.empty_like(x)
    y.copy_(x)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(20):
        y.copy_(x)
    e1.record()
    torch.cuda.synchronize()
    copy_gbs = 2.0 * x.numel() * 2 * 20 / (e0.elapsed_time(e1) / 1000.0) / 1e9
    del a, b, c, x, y
    return {"gemm": "torch.matmul fp16 4096^3, seeded random", "gemm_reps": reps, "gemm_us": round(gemm_us, 2),
            "gemm_tflops": round(2 * 4096 ** 3 / (gemm_us * 1e-6) / 1e12, 1), "copy_gbs": round(copy_gbs, 1)}


def cpu_baseline(cfg, ws, ms, vs, seconds, speedup, threads, hs=None, fast=True, host=None):
    """The oracle (CPU restatement of the reference path, torch-CPU fp32) on ONE clip of the same
    workload, timed on this host: mel/energy, F0, pitch shift, Whisper-medium, map, conditioner,
    PLMS (speedup 10 = 101 denoiser calls), de-normalisation, BigVGAN, fade."""
    from oracle import pipeline as OP
    torch.set_num_threads(threads)
    host = dict(host or {})
    w24, w16 = synth_inputs([0], seconds, float16k=hs is not None)
    if fast:
        t0 = time.time()
        OP.convert(cfg, ws, ms, vs, w24[0], w16[0], singer=1, speedup=speedup, seed=0, hs=hs)
        dt = time.time() - t0
        return {"value": round(seconds / dt, 4), "unit": "audio-s/s", "cores": threads, "kind": "port", **host,
                "sample": f"1 x {seconds:g} s clip, full oracle path (PLMS speedup {speedup}), torch-CPU fp32, "
                          f"{threads} threads (all CPUs available to the process), {dt:.1f} s"}
    # DDPM-1000 on the CPU is ~2 min per clip: time the path once with PLMS speedup 250 (5 denoiser calls) and
    # 10 more denoiser calls alone, then extrapolate the sampler to 1000 calls.
    from oracle import models as OM
    t0 = time.time()
    OP.convert(cfg, ws, ms, vs, w24[0], w16[0], singer=1, speedup=250, seed=0, hs=hs)
    t_path = time.time() - t0
    T = (w24.shape[1] + 768 - 1024) // 256 + 1
    cond = torch.randn(1, T, cfg.mapper.residual_channels)
    x = torch.randn(1, T, cfg.mapper.n_mel)
    table = W.step_embedding_table(1000)
    t0 = time.time()
    for i in range(10):
        OM.diffsvc_forward(ms, cfg.mapper, x, cond, torch.tensor([999 - i]), table)
    t_call = (time.time() - t0) / 10
    dt = t_path + (1000 - 5) * t_call
    return {"value": round(seconds / dt, 4), "unit": "audio-s/s", "cores": threads, "kind": "port", **host,
            "sample": f"1 x {seconds:g} s clip, oracle path with 5 denoiser calls ({t_path:.1f} s) + 995 x "
                      f"{t_call * 1e3:.0f} ms timed denoiser calls (DDPM-1000 extrapolated), torch-CPU fp32, {threads} threads"}


# algorithmic FLOPs of one 10 s clip (T = 937 mel frames) per component; the frame-proportional parts
# scale with T, Whisper / HuBERT run on their fixed 30 s / 10 s input
SURVEY_TF = {"whisper": 1.138, "contentvec": 0.128, "cond": 0.0007 + 0.011, "denoise_call": 0.04464, "bigvgan": 1.718}


def survey_algorithmic_tflops(clips, T, calls, content="whisper"):
    """§8(d)'s algorithmic work of a step (TFLOP): the reference's model FLOPs, without the split-fp16 / weight-split
    duplicate MFMA work this build executes for precision (reported separately as executed_tflops_per_step)."""
    r = T / 937.0
    return clips * (SURVEY_TF[content] + r * (SURVEY_TF["cond"] + calls * SURVEY_TF["denoise_call"] +
                                              SURVEY_TF["bigvgan"]))


def family(prof):
    """{"kernel@site": rec} -> {kernel: summed rec}"""
    out = {}
    for name, v in prof.items():
        agg = out.setdefault(name.split("@")[0], dict(ms=0.0, launches=0, flops=0.0, bytes=0.0))
        for f in agg:
            agg[f] += v[f]
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv):
    """Run `bench.py argv` as n rank processes (RANK = LOCAL_RANK = 0..n-1, WORLD_SIZE = n, rendezvous on
    127.0.0.1) and return the worst exit status. The caller has not touched the GPU (no torch.cuda call, no
    libsvc_hip load): every rank is a fresh child process, nothing is exec'ed from a GPU-initialised process."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    # poll all ranks: the first failure ends the others (a peer blocked in a collective would never return)
    rc = 0
    while any(p.poll() is None for p in procs):
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad:
            rc = bad[0] if bad[0] > 0 else 128 - bad[0]
            for p in procs:
                if p.poll() is None:
                    p.kill()
            break
        time.sleep(0.2)
    for p in procs:
        code = p.wait()
        if code != 0 and rc == 0:
            rc = code if code > 0 else 128 - code
    return rc


def dry_run(args, dist):
    """CPU stand-in for the engine (gloo): each rank "converts" its shard of synthetic clips by the identity
    (the 24 kHz clip trimmed to T*hop samples, as the vocoder output is), keyed by global utterance id exactly as
    the GPU run is, then runs the same gather. Rank 0 prints the bench line's distributed fields and, with
    --dump, saves the gathered waveforms, so world 1 and world N outputs can be compared (tests/test_parallel.py)."""
    B = args.batch
    uids = np.arange(dist.rank * B, (dist.rank + 1) * B)
    w24, _ = synth_inputs(uids, args.seconds)
    T = (w24.shape[1] + 768 - 1024) // 256 + 1
    wav = torch.from_numpy(np.ascontiguousarray(w24[:, :T * 256]))
    dist.barrier()
    t0 = time.time()
    out = None
    gather_s = []
    for i in range(args.steps):
        if args.fault and dist.rank == args.fault_rank and i == min(1, args.steps - 1):
            # fault injection (tests/test_parallel.py): this rank fails mid-run, by an exception or by hanging
            # without exiting; the peers must not wait forever in the gather
            if args.fault == "raise":
                raise RuntimeError(f"injected fault on rank {dist.rank} at step {i}")
            time.sleep(3600)
        tg = time.perf_counter()
        out, lens = dist.gather_waveforms(wav, return_lengths=True)
        gather_s.append(time.perf_counter() - tg)
    dist.barrier()
    per_rank = [r[0] for r in dist.all_gather_floats([time.time() - t0])]
    gather_ms = [r[0] for r in dist.all_gather_floats([1000.0 * sum(gather_s) / max(len(gather_s), 1)])]
    elapsed = max(per_rank)
    if dist.rank == 0:
        assert out.shape[0] == dist.world * B and bool(torch.isfinite(out).all())
        if args.dump:
            np.save(args.dump, out.numpy())
        print(json.dumps({"metric": "dry-run gather (identity conversion, CPU)", "n_gpus": args.gpus,
                          "dist_world": dist.world, "backend": dist.backend or "none",
                          "rccl_world": torchdist.get_world_size() if torchdist.is_initialized() else 1,
                          "gather_ms_per_step": [round(v, 3) for v in gather_ms], "steps": args.steps,
                          "per_rank_s": [round(t, 4) for t in per_rank], "elapsed_s": round(elapsed, 4),
                          "gathered": list(out.shape), "lengths": lens.tolist()}), flush=True)
    dist.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo identity conversion: exercises the rank spawn, sharding and gather only")
    ap.add_argument("--dump", default=None, help="(--dry-run) save rank 0's gathered waveforms to this .npy")
    ap.add_argument("--fault", choices=["raise", "hang"], default=None,
                    help="(--dry-run) rank --fault-rank raises / hangs at the second step (failure-path tests)")
    ap.add_argument("--fault-rank", type=int, default=1)
    ap.add_argument("--dist-timeout", type=float, default=None,
                    help="collective timeout in seconds (default SVC_DIST_TIMEOUT_S or 600)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32, help="clips per GPU")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--speedup", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-calib", action="store_true", help="skip the box-speed calibration GEMM / copy")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads for the CPU baseline (default: every CPU available to the process)")
    ap.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    ap.add_argument("--no-isolated-pass", action="store_true",
                    help="skip the untimed single-stream pass of the dominant call site (profiling runs: every launch "
                         "of the dominant kernel in the trace is then a production launch)")
    ap.add_argument("--content", choices=["whisper", "contentvec"], default="whisper",
                    help="content encoder (BASELINE config 5: contentvec = the HuBERT/ContentVec variant)")
    ap.add_argument("--sampler", choices=["plms", "ddpm"], default="plms",
                    help="plms = the reference's fast_inference PLMS (speedup --speedup); ddpm = 1000-step DDPM")
    ap.add_argument("--precision", choices=["wsplit", "split", "fp16"], default="wsplit",
                    help="wsplit (default): weight-split Whisper attention linears (every block) and MLP linears "
                         "(blocks 0-3), split-fp16 conv stem / HuBERT / DiffSVC head, the mode that meets the 1e-3 "
                         "mel-L1 target (tests/test_gpu_headline.py); split: every content GEMM on split-fp16 "
                         "operands; fp16: plain fp16 operands (faster, fails the target)")
    ap.add_argument("--operands", choices=["fp16", "bf16"], default="fp16",
                    help="16-bit MFMA operand format of the content encoder, conditioner and DiffSVC GEMMs (BigVGAN "
                         "stays fp16); bf16 = BASELINE configs[4]'s variant, which does not meet the mel-L1 target")
    ap.add_argument("--wsplit-mlp", type=int, default=None,
                    help="wsplit: bit mask of the Whisper blocks whose MLP linears are weight-split (default 0xf; "
                         "16777215 = all 24, the round-2 default before the precision sweep)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}")
    if args.dry_run:
        return dry_run(args, DistContext.from_env(backend="gloo", timeout_s=args.dist_timeout))

    dist = DistContext.from_env(timeout_s=args.dist_timeout)
    torch.cuda.set_device(dist.local_rank)
    cfg = C.load_config()
    t_setup = time.time()
    ws = hs = None
    if args.content == "whisper":
        ws = W.make_whisper_state(W.WHISPER_DIMS["medium"], seed=0)
    else:
        cfg.mapper.content_feature = ["contentvec"]
        cfg.mapper.input_content_dim["contentvec"] = W.HUBERT_DIMS["contentvec"]["final_dim"]
        hs = W.make_hubert_state(W.HUBERT_DIMS["contentvec"], seed=0)
    ms = W.make_mapper_state(cfg.mapper, seed=0)
    vs = W.make_vocoder_state(cfg.vocoder, seed=0)
    eng = SVCEngine(cfg, dist.local_rank, whisper_state=ws, mapper_state=ms, vocoder_state=vs, hubert_state=hs,
                    content_split={"split": 1, "wsplit": 2, "fp16": 0}[args.precision],
                    head_split=args.precision != "fp16",
                    config=None if args.wsplit_mlp is None else {"content.wsplit_mlp": args.wsplit_mlp},
                    operands=args.operands)
    fast = args.sampler == "plms"
    pipe = SVCPipeline(eng)
    B = args.batch
    uids = np.arange(dist.rank * B, (dist.rank + 1) * B)
    w24, w16 = synth_inputs(uids, args.seconds, float16k=args.content == "contentvec")
    d24 = torch.from_numpy(w24).cuda()
    d16 = torch.from_numpy(w16).cuda()
    singer = torch.from_numpy((uids % 5).astype(np.int32)).cuda()
    utt = torch.from_numpy(uids.astype(np.int32)).cuda()
    log(f"rank {dist.rank}/{dist.world}: setup {time.time() - t_setup:.1f}s, weights {eng.memory()[0] / 1e9:.2f} GB")

    gather_s = []  # the RCCL gather's own wall time per step (convert finished first: synchronized on both sides)

    def step():
        res = pipe.convert(d24, d16, singer, fast_inference=fast, speedup=args.speedup, seed=1234, utt_ids=utt,
                           wav16_float=d16 if hs is not None else None)
        torch.cuda.synchronize()
        tg = time.perf_counter()
        out = dist.gather_waveforms(res.wav)
        torch.cuda.synchronize()
        gather_s.append(time.perf_counter() - tg)
        return out

    # Warmup. The last warmup step runs with every launch profiled (HIP events around each kernel): that
    # gives the per-kernel breakdown and picks the dominant kernel. The timed steps then record events
    # only around that kernel's launches (svc_profile_filter), so the roofline is measured live in the
    # timed region without bracketing the other ~4 000 launches per step.
    prof_all = {}
    for i in range(max(args.warmup, 1)):
        last = i == max(args.warmup, 1) - 1
        if last:
            _lib.profile_enable(True)
        step()
        torch.cuda.synchronize()
        if last:
            prof_all = _lib.profile_read()
            _lib.profile_enable(False)
        log(f"warmup {i + 1}/{args.warmup}")

    by_kernel = family(prof_all)
    dom_name = max(by_kernel.items(), key=lambda kv: kv[1]["ms"])[0]
    share = by_kernel[dom_name]["ms"] / sum(v["ms"] for v in by_kernel.values())
    dom_site = max((n for n in prof_all if n.split("@")[0] == dom_name), key=lambda n: prof_all[n]["ms"])
    dom_site = dom_site.split("@")[1] if "@" in dom_site else ""

    # The sampler runs utterance-aligned sub-batches on concurrent streams (kernel switch sampler_streams, read back
    # from the library), so a launch's HIP-event duration includes time shared with the other streams' kernels. One
    # extra untimed step with the sampler on a single stream gives the dominant call site's isolated per-launch rate.
    streams = int(eng.get_config("tune.sampler_streams"))
    isolated = None
    if streams > 1 and dom_site.startswith("diffsvc.") and not args.no_isolated_pass:
        eng.tune(sampler_streams=1)
        _lib.profile_enable(True)
        step()
        torch.cuda.synchronize()
        iso = _lib.profile_read()
        _lib.profile_enable(False)
        eng.tune(sampler_streams=streams)
        at_site = {n.split("@")[0]: v for n, v in iso.items() if n.endswith("@" + dom_site)}
        if at_site:
            k, v = max(at_site.items(), key=lambda kv: kv[1]["ms"])
            us = v["ms"] * 1000.0 / v["launches"]
            tf = v["flops"] / v["launches"] / (us * 1e-6) / 1e12
            isolated = {"kernel": k, "site": dom_site, "avg_launch_us": round(us, 2), "achieved": round(tf, 2),
                        "frac": round(tf / PEAK_F16_TFLOPS, 4), "sampler_streams": 1, "launches": v["launches"]}

    # The timed steps run with no HIP events at all: one extra untimed production step after them (same configuration,
    # every launch of the dominant kernel between its own event pair) gives the roofline's per-launch figures. Event
    # pairs around the ~2 000 gate launches per step cost 2 % of the step (r04m: 866.4 / 867.6 with them against
    # 884.4 / 883.4 audio-s/s without, alternating); BENCH_TIMED_EVENTS=1 puts them back into the timed region.
    timed_events = os.environ.get("BENCH_TIMED_EVENTS", "0") == "1"
    dist.barrier()
    torch.cuda.synchronize()
    if timed_events:
        _lib.profile_filter(dom_name)
        _lib.profile_enable(True)
    gather_s.clear()
    clocks = ClockSampler(dist.local_rank)
    clocks.start()
    t0 = time.time()
    for i in range(args.steps):
        out = step()
        torch.cuda.synchronize()
        log(f"step {i + 1}/{args.steps} {time.time() - t0:.2f}s")
    torch.cuda.synchronize()
    dist.barrier()
    per_rank = [r[0] for r in dist.all_gather_floats([time.time() - t0])]
    clocks.stop()
    gather_ms = [r[0] for r in dist.all_gather_floats([1000.0 * sum(gather_s) / max(len(gather_s), 1)])]
    elapsed = max(per_rank)
    if not timed_events:
        _lib.profile_filter(dom_name)
        _lib.profile_enable(True)
        step()
        torch.cuda.synchronize()
    prof = _lib.profile_read()
    _lib.profile_enable(False)
    _lib.profile_filter("")
    ms_per_step = 1000.0 * elapsed / args.steps
    audio_s = dist.world * B * args.seconds
    value = audio_s / (elapsed / args.steps)
    if out is not None:
        assert out.shape[0] == dist.world * B and bool(torch.isfinite(out).all())

    # Roofline of the dominant kernel AS THE TIMED REGION RUNS IT (its production launches: at a diffsvc.* site the
    # sampler's utterance-aligned sub-batches on `streams` concurrent streams), HIP events around each launch on its
    # launch stream. A launch's event span then includes time its waves share the CUs with the other stream's kernels
    # (and the event markers' own gap); rocprof's per-dispatch duration of the same launches, from the
    # committed profile of record, stands beside it, and so does the untimed single-stream pass (full batch per launch).
    dom = dict(ms=0.0, launches=0, flops=0.0, bytes=0.0)
    for name, v in prof.items():
        if name.split("@")[0] == dom_name:
            for f in dom:
                dom[f] += v[f]
    per_launch_s = dom["ms"] / 1000.0 / dom["launches"]
    if dom["flops"] > 0:
        achieved = dom["flops"] / dom["launches"] / per_launch_s / 1e12
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s"}
    else:
        achieved = dom["bytes"] / dom["launches"] / per_launch_s / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s"}
    roof["frac"] = round(roof["achieved"] / roof["peak"], 4)
    roof["kernel"] = dom_name
    roof["site"] = dom_site
    roof["avg_launch_us"] = round(per_launch_s * 1e6, 2)
    roof["launches_timed"] = dom["launches"]
    roof["algorithmic_per_launch"] = round(dom["flops"] / dom["launches"] if dom["flops"] > 0 else
                                           dom["bytes"] / dom["launches"], 1)
    roof["share_of_kernel_time"] = round(share, 3)
    roof["sampler_streams"] = streams
    T_frames = int((d24.shape[1] + 768 - 1024) // 256 + 1)
    if dom_site.startswith("diffsvc."):
        roof["rows_per_launch"] = -(-B // streams) * T_frames  # the largest sub-batch
    roof["measured"] = ("production launches in the timed region, HIP events on the launch stream" if timed_events else
                        "production launches of one untimed step right after the timed region (the timed steps run "
                        "without events), HIP events on the launch stream")
    if isolated:
        roof["isolated_single_stream"] = {k: isolated[k] for k in ("kernel", "avg_launch_us", "achieved", "launches")}
        roof["isolated_single_stream"]["frac"] = isolated["frac"]
        roof["isolated_single_stream"]["rows_per_launch"] = B * T_frames
        roof["isolated_single_stream"]["measured"] = ("untimed single-stream pass of the dominant call site (full "
                                                      "batch per launch), HIP events on the launch stream")
    # committed profile of record (tools/gpu_profile.sh: rocprofv3 trace + separate FETCH_SIZE / WRITE_SIZE passes of
    # bench.py --no-isolated-pass, so every dispatch of the kernel there is a production launch)
    roof["traffic"] = None
    # the committed PMC / rocprof records are of the headline configuration (configs[1]); other workloads (e.g. the 180 s
    # song) launch the kernel on other shapes, so those records do not describe their launches
    headline_cfg = (B == 32 and args.seconds == 10.0 and args.content == "whisper" and fast and args.speedup == 10)
    if not headline_cfg:
        roof["traffic_source"] = "not measured for this workload (the PMC records are of configs[1])"
    if headline_cfg and os.path.exists(args.pmc_json):
        pmc = json.load(open(args.pmc_json))
        ent = pmc.get("kernels", {}).get(dom_name)
        if ent:
            roof["traffic"] = ent.get("hbm_bytes_per_launch")
            src = os.path.relpath(args.pmc_json, REPO) + " (" + pmc.get("source_run", "?") + \
                (f", {ent['workgroups']}-workgroup launches" if "workgroups" in ent else "") + ")"
            roof["traffic_source"] = src
            if "rocprof_trace_avg_us" in ent:
                roof["rocprof_avg_launch_us"] = round(ent["rocprof_trace_avg_us"], 2)
                if dom["flops"] > 0:
                    roof["rocprof_achieved"] = round(dom["flops"] / dom["launches"] /
                                                     (ent["rocprof_trace_avg_us"] * 1e-6) / 1e12, 2)
                    roof["rocprof_frac"] = round(roof["rocprof_achieved"] / PEAK_F16_TFLOPS, 4)
    # MFMA utilisation of the roofline kernel's production grid from the serialised PMC passes (tools/pmc_kernels.sh):
    # SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE x 1024 SIMDs, per dispatch
    pmc_k = os.path.join(os.path.dirname(args.pmc_json), "pmc_kernels.json")  # latest tools/pmc_kernels.sh summary
    if headline_cfg and os.path.exists(pmc_k):
        ents = [v for v in json.load(open(pmc_k)).values() if v.get("kernel") == dom_name and "mfma_busy" in v]
        if ents:
            big = max(ents, key=lambda v: v.get("dispatches", 0))  # the production grid has the most dispatches
            roof["mfma_busy_pmc"] = round(big["mfma_busy"], 3)
            if "valu_per_mfma" in big:
                roof["valu_per_mfma_pmc"] = round(big["valu_per_mfma"], 2)
            roof["mfma_busy_source"] = os.path.relpath(pmc_k, REPO) + f" ({big['workgroups']}-workgroup launches)"
    # per-kernel breakdown of the fully profiled warmup step
    total_flops = sum(v["flops"] for v in prof_all.values())
    calls = (1000 // args.speedup + 1) if fast else 1000
    alg_tf = survey_algorithmic_tflops(dist.world * B, T_frames, calls,
                                       "whisper" if hs is None else "contentvec")
    kernels = {k: {"ms_per_step": round(v["ms"], 3), "launches_per_step": v["launches"],
                   "tflops": round(v["flops"] / max(v["ms"], 1e-9) / 1e9, 1) if v["flops"] else None,
                   "gbs": round(v["bytes"] / max(v["ms"], 1e-9) / 1e6, 1) if v["bytes"] else None}
               for k, v in sorted(prof_all.items(), key=lambda kv: -kv[1]["ms"])}

    calib = None
    if not args.no_calib:
        try:
            calib = calibrate(dist.local_rank)
        except Exception as e:  # noqa: BLE001 (reported, never fatal)
            calib = {"error": f"{type(e).__name__}: {e}"}
    cpu = None
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        log("cpu baseline (oracle, 1 clip)...")
        threads, host = host_cpus()
        cpu = cpu_baseline(cfg, ws, ms, vs, args.seconds, args.speedup, args.cpu_threads or threads, hs=hs,
                           fast=fast, host=host)
    if dist.rank == 0:
        line = {
            "metric": "converted audio sec/sec (RTF^-1) end-to-end, 10 s clips",
            "value": round(value, 2), "unit": "audio-s/s", "n_gpus": dist.world, "steps": args.steps,
            "dist_world": dist.world, "backend": dist.backend or "none",
            # the process group's own size (torch.distributed.get_world_size(); 1 without a group) and the gather's
            # wall time per step on each rank (rank 0 receives; world 1: no collective)
            "rccl_world": torchdist.get_world_size() if torchdist.is_initialized() else 1,
            "gather_ms_per_step": [round(v, 3) for v in gather_ms],
            "per_rank_ms_per_step": [round(1000.0 * t / args.steps, 2) for t in per_rank],
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.operands, "data": "synthetic",
            "config": {"workload": f"batch={B}/GPU x {args.seconds:g} s synthetic clips, "
                                   + ("Whisper-medium" if hs is None else "HuBERT/ContentVec (layer 9)")
                                   + (f" + PLMS-100 DiffSVC (speedup {args.speedup})" if fast else " + DDPM-1000 DiffSVC")
                                   + f" + BigVGAN, {args.operands} MFMA operands (BigVGAN fp16) / fp32 accumulate"
                                   + {"split": ", split-fp16 content encoder + DiffSVC head (mel-L1 <= 1e-3 mode)",
                                      "wsplit": ", weight-split Whisper attention linears (all blocks) + MLP linears "
                                                "(blocks 0-3) + split-fp16 stem / DiffSVC head",
                                      "fp16": ", plain fp16 operands (mel-L1 target not met)"}[args.precision],
                       "global_batch": dist.world * B, "seq_len_frames": int((d24.shape[1] + 768 - 1024) // 256 + 1),
                       "parallelism": f"dp{dist.world} (per-utterance shards, RCCL gather)"},
            "roofline": roof, "cpu_baseline": cpu,
            # box speed beside the value: rank 0's GPU clocks sampled through the timed region, and a fixed hipBLASLt
            # GEMM / HBM copy calibration timed in this process after it (calib_us = that GEMM's time per launch)
            "clocks": clocks.summary(), "calib": calib, "calib_us": calib.get("gemm_us") if calib else None,
            # SURVEY.md §8(d) algorithmic work (the reference's model FLOPs) and the end-to-end fraction of the MFMA
            # peak it sustains; executed_* counts the MFMA work actually issued (split-fp16 / weight-split duplicates)
            "algorithmic_tflops_per_step": round(alg_tf, 2),
            "sustained_tflops": round(alg_tf / (ms_per_step / 1000.0), 1),
            "sustained_frac": round(alg_tf / (ms_per_step / 1000.0) / PEAK_F16_TFLOPS, 4),
            "executed_tflops_per_step": round(total_flops * dist.world / 1e12, 2),
            "executed_sustained_tflops": round(total_flops * dist.world / 1e12 / (ms_per_step / 1000.0), 1),
            "kernels_profiled_step": "last warmup step, every launch bracketed by HIP events (sampler sub-batches on "
                                     f"{streams} concurrent streams: their per-launch times overlap)",
            "kernels": kernels,
        }
        print(json.dumps(line), flush=True)
    dist.close()


if __name__ == "__main__":
    main()
