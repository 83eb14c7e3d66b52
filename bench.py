"""Benchmark: train frames/s of the 228M NeuroSync Seq2Seq on MI355X (BASELINE.json metric).

One step = one reference training step (utils/training_utils.py:56-80) on one
batch of B=128 windows x T=128 frames per GPU: zero_grad -> forward -> fused
Loss -> backward -> clip(2.0) + Adam; when n>1 the optimizer is sharded
(RCCL reduce-scatter of the gradients, Adam on 1/n, all-gather of the weights).
bf16 compute, dropout 0.3 on, synthetic seeded inputs of the reference shapes
(features [B,T,256] f32, targets [B,T,61] f32, already resident in HBM).

  python bench.py [--gpus N --steps K --warmup W]

N>1: started as `python bench.py --gpus N`, this process touches no GPU and
runs `python -m torch.distributed.run --nnodes 1 --nproc-per-node N
--master-addr 127.0.0.1 ... bench.py ...` as a child, relaying rank 0's line
(launch_ranks); started by torchrun itself (WORLD_SIZE set), it is one rank, and
WORLD_SIZE must equal --gpus.  Under the self-launch, a first attempt with the
default exchange (NSTL_DP=zero1_push) that fails or stalls is followed by one
with NSTL_DP=zero1, and the line records both (`launch.attempts`).

Multi-rank lines also carry `dist` (backend, world size, launch form, per-rank
ms/step and their spread, and `exchange_check`: the first step's pushed shard
sums against an RCCL reduce-scatter, ShardPusher.verify), `config.gradient_exchange`
(the exchange active after the timed steps) and `config.dp_fallback`.

Prints ONE JSON line on rank 0.  `roofline` is measured live for the dominant
kernel (nstl GEMM: ~97% of the step's FLOPs): HIP events around every GEMM launch
of the last --gemm-sample-steps timed steps (events on all ~270 launches of every
step would add ~1.7 ms/step), on the stream it runs on; achieved = algorithmic
GEMM FLOPs / GEMM time.  `cpu_baseline` times the fp32 CPU oracle step (the reference step
restated in torch-CPU) on a bounded sample on rank 0.  `parity` is the metric's
"MSE vs ref": forward output of the full 228M config vs the fp32 CPU oracle on
the same 2-window batch and seeded weights (fp32 mode gated at 1e-3; bf16 reported).
--fp8 is BASELINE config C5 (e4m3 attention q/k/v + encoder FFN1 forward GEMMs; add --seq 256
--batch 64 for its doubled clip length): its fp8 GEMM launches are reported as
`roofline_fp8` against the fp8 dense peak, and `parity` adds the fp8 forward MSE.
"""
import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

BF16_DENSE_PEAK_TFLOPS = 2516.6  # 256 CU x 2.4 GHz x 4096 FLOP/clk/CU (MI355X_MICROARCH.md)
FP8_DENSE_PEAK_TFLOPS = 5033.2   # scaled f8f6f4 MFMA: 2x bf16 per clock (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def log(msg):
    print("[bench] " + msg, file=sys.stderr, flush=True)


def frames_flops(W, T, D, n_attn=24):
    """Algorithmic train FLOPs per frame: 6W + 12*T*D*24."""
    return 6 * W + 12 * T * D * n_attn


def _is_bf16_gemm(name):
    # every hand-written bf16 GEMM kernel: the same launches the in-run HIP-event
    # timing of nstl_gemm / nstl_gemm_grouped sees
    return "gemm" in name and "splitk" not in name and "f8" not in name


# GEMM families for the per-family split of traffic and MFMA busy (kernel names
# as rocprofv3 reports them, demangled)
def _gemm_family(name):
    if "gemm4_kernel" in name:
        # template <AK, BKM, EM, GROUPED, DBG>: the grouped weight gradients are <false, false, 5, true
        return "gemm4_grouped_dw" if "<false, false, 5, true" in name else "gemm4"
    if "gemm256r" in name or "gemm256_kernel" in name:
        return "ring"
    return "gemm128"


def _pmc_dispatches(d):
    """{dispatch id: (kernel name, ns, {counter: summed value})} of a rocprofv3
    --output-format csv counter run."""
    import csv
    import glob
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = int(r["Dispatch_Id"])
            if k not in out:
                out[k] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), {})
            c = out[k][2]
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def measure_gemm_counters(args):
    """PMC figures of the GEMM family, measured on this box in this run by three
    rocprofv3 counter passes over a child run of this same bench (1 warm-up + 1
    step of the same workload), started before this process touches the GPU:
      - FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH.md): HBM
        bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) KiB * 1024 (gfx950
        FETCH_SIZE counts streaming reads at half their bytes);
      - SQ_VALU_MFMA_BUSY_CYCLES with GRBM_GUI_ACTIVE: the share of the clock
        cycles the matrix pipes were busy, MFMA / (GRBM_GUI_ACTIVE / 8 XCDs x 1024
        SIMDs), and the clock the kernel ran at (GRBM_GUI_ACTIVE / 8 / wall).
    Returns {"traffic": bytes|None, "note": str, "mfma_busy": {...}|None}."""
    import shutil
    import subprocess
    import tempfile
    res = {"traffic": None, "mfma_busy": None}
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        res["note"] = "rocprofv3 absent: counters not measured"
        return res
    runs = {}
    t0 = time.perf_counter()
    for tag, counters in (("FETCH_SIZE", ["FETCH_SIZE"]), ("WRITE_SIZE", ["WRITE_SIZE"]),
                          ("MFMA", ["SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"])):
        d = tempfile.mkdtemp(prefix="nstl_pmc_", dir="/tmp")
        cmd = ["timeout", "-s", "KILL", "240", exe, "--pmc"] + counters + [
               "-d", d, "-o", "run", "--output-format", "csv",
               "--", sys.executable, os.path.abspath(__file__), "--steps", "1", "--warmup", "1", "--no-cpu-baseline",
               "--no-parity", "--feature-steps", "0", "--feed-steps", "0", "--no-traffic",
               "--batch", str(args.batch), "--seq", str(args.seq)] + (["--fp8"] if args.fp8 else []) + \
              (["--fp8-bwd"] if args.fp8_bwd else [])
        env = dict(os.environ, TMPDIR="/tmp")
        log("counters: rocprofv3 --pmc %s pass (child bench, 1+1 steps)" % " ".join(counters))
        r = subprocess.run(cmd, env=env, cwd="/tmp", stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
        if r.returncode != 0:
            log("counters: %s pass failed (rc %d): %s" % (tag, r.returncode, r.stderr[-400:]))
            res["note"] = "rocprofv3 %s pass failed (rc %d): counters not measured" % (tag, r.returncode)
            return res
        runs[tag] = _pmc_dispatches(d)
        shutil.rmtree(d, ignore_errors=True)
    log("counters: three passes in %.1fs" % (time.perf_counter() - t0))
    kib = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        v = [x[2][c] for x in runs[c].values() if _is_bf16_gemm(x[0]) and c in x[2]]
        if not v:
            res["note"] = "rocprofv3 %s pass recorded no GEMM dispatch: traffic not measured" % c
            return res
        kib[c] = sum(v) / len(v)
    res["traffic"] = round((2.0 * kib["FETCH_SIZE"] + kib["WRITE_SIZE"]) * 1024.0)
    # the same per GEMM family (bytes per launch, mean over the family's dispatches)
    fam = {}
    for f in ("gemm4", "gemm4_grouped_dw", "ring", "gemm128"):
        per = {}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            v = [x[2][c] for x in runs[c].values() if _is_bf16_gemm(x[0]) and _gemm_family(x[0]) == f and c in x[2]]
            per[c] = (sum(v) / len(v), len(v)) if v else None
        if per["FETCH_SIZE"] and per["WRITE_SIZE"]:
            fam[f] = {"traffic": round((2.0 * per["FETCH_SIZE"][0] + per["WRITE_SIZE"][0]) * 1024.0),
                      "dispatches": per["FETCH_SIZE"][1]}
    res["traffic_by_family"] = fam
    res["note"] = ("measured in this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over a 1+1-step child run of "
                   "this workload, mean over its bf16 GEMM-family dispatches")

    def busy(sel):
        xs = [x for x in runs["MFMA"].values() if sel(x[0]) and "GRBM_GUI_ACTIVE" in x[2]]
        if not xs:
            return None
        grbm = sum(x[2]["GRBM_GUI_ACTIVE"] for x in xs)
        mfma = sum(x[2].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for x in xs)
        ns = sum(x[1] for x in xs)
        return {"mfma_busy": round(mfma / (grbm / 8 * 1024), 4), "clock_ghz": round(grbm / 8 / ns, 3),
                "dispatches": len(xs)}
    res["mfma_busy"] = {"gemm_family": busy(_is_bf16_gemm),
                        "grouped_dw": busy(lambda n: _is_bf16_gemm(n) and _gemm_family(n) == "gemm4_grouped_dw"),
                        "by_family": {f: busy(lambda n, f=f: _is_bf16_gemm(n) and _gemm_family(n) == f)
                                      for f in ("gemm4", "gemm4_grouped_dw", "ring", "gemm128")},
                        "source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE, child run (1+1 steps); "
                                  "busy = MFMA cycles / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs); profiled runs "
                                  "clock a few % below un-profiled ones"}
    return res


def cpu_baseline(cfg, T, budget_s=20.0):
    """fp32 oracle step (reference semantics) on the host cores, bounded sample."""
    from oracle import model_ref
    # the GPU box's affinity mask shows the whole machine; the job's CPU share is
    # what OMP_NUM_THREADS says there (16)
    cores = len(os.sched_getaffinity(0))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        cores = min(cores, int(os.environ["OMP_NUM_THREADS"]))
    torch.set_num_threads(cores)
    B = 8  # the CPU sample is B=8 windows x T frames
    params = model_ref.seeded_params(model_ref.param_shapes(cfg["input_dim"], cfg["hidden_dim"], cfg["n_layers"],
                                                            cfg["output_dim"]), 0)
    tr = model_ref.OracleTrainer(params, cfg["num_heads"], dropout=cfg["dropout"])
    g = torch.Generator().manual_seed(0)
    src = torch.randn(B, T, cfg["input_dim"], generator=g)
    trg = torch.randn(B, T, cfg["output_dim"], generator=g) * 20
    t0 = time.perf_counter()
    tr.step(src, trg)  # warm-up
    log("cpu baseline warm-up step %.1fs (%d threads)" % (time.perf_counter() - t0, cores))
    n, t0 = 0, time.perf_counter()
    while n < 3 or time.perf_counter() - t0 < budget_s:
        tr.step(src, trg)
        n += 1
        log("cpu baseline step %d done at %.1fs" % (n, time.perf_counter() - t0))
    dt = time.perf_counter() - t0
    return {"value": round(n * B * T / dt, 2), "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": "228M fp32 oracle step (fwd+loss+bwd+clip+Adam, dropout 0.3), B=%d x T=%d frames, %d timed steps"
                      % (B, T, n)}


def synth_corpus(root, clips, seconds, seed=0, sr=88200, fps=60):
    """BASELINE C4's corpus, synthetic and seeded: per clip a
    folder with an 88.2 kHz 16-bit mono WAV (3 harmonics of f0 ~ U[80, 300] Hz,
    4 Hz AM, N(0, 0.01^2) noise, peak-normalised) and a 60 fps
    *_iPhone_cal.csv of 61 blendshape/pose curves (low-pass noise: cols 0-51
    clipped to [0, 1], cols 52-60 0.3 tanh) -- the files process_folder reads."""
    import numpy as np
    import pandas as pd
    from neurosync_trainer_lite_amd.utils.audio.load_audio import write_wav
    from neurosync_trainer_lite_amd.utils.csv.save_csv import BLENDSHAPE_COLUMNS
    rng = np.random.default_rng(seed)
    n, nf = int(seconds * sr), int(seconds * fps)
    t = np.arange(n) / sr
    k = np.exp(-np.arange(-30, 31) ** 2 / (2 * 8.0 ** 2))
    k /= k.sum()
    for c in range(clips):
        d = os.path.join(root, "clip%03d" % c)
        os.makedirs(d, exist_ok=True)
        f0 = rng.uniform(80, 300)
        y = sum((0.6 / h) * np.sin(2 * np.pi * h * f0 * t + rng.uniform(0, 6.28)) for h in (1, 2, 3))
        y = y * (0.55 + 0.45 * np.sin(2 * np.pi * 4 * t)) + 0.01 * rng.standard_normal(n)
        write_wav(os.path.join(d, "audio.wav"), (y / np.abs(y).max()).astype(np.float32), sr)
        z = np.stack([np.convolve(rng.standard_normal(nf), k, mode="same") for _ in range(61)], 1) * 4
        z[:, :52] = np.clip(z[:, :52], 0, 1)
        z[:, 52:] = 0.3 * np.tanh(z[:, 52:])
        df = pd.DataFrame(z, columns=BLENDSHAPE_COLUMNS)
        df.insert(0, "BlendshapeCount", 61)
        df.insert(0, "Timecode", ["%02d:%02d:%02d:%02d.000" % (i // 216000, i // 3600 % 60, i // 60 % 60, i % 60)
                                  for i in range(nf)])
        df.to_csv(os.path.join(d, "take_iPhone_cal.csv"), index=False)


def data_feed(cfg, args, step_fn, dev, rank, world):
    """BASELINE C4's feed: the synthetic corpus through the drop-in data path
    (prepare_dataloader_with_split -> load_data -> collect_features with
    include_fast + include_slow -> GPU feature extraction -> windows), batches
    fetched whole into pinned host memory and copied with non_blocking H2D into
    the same train step; rank r of n takes batches r, r+n, ... (rank_batches)."""
    import contextlib
    import tempfile
    from neurosync_trainer_lite_amd.dataset.dataset import prepare_dataloader_with_split
    from neurosync_trainer_lite_amd.utils.training_utils import rank_batches
    t0 = time.perf_counter()
    # the data path prints its progress as the reference does: keep stdout for the JSON line
    with tempfile.TemporaryDirectory(prefix="nstl_c4_%d_" % rank) as root, contextlib.redirect_stdout(sys.stderr):
        synth_corpus(root, args.feed_clips, args.feed_seconds, seed=0)
        c = dict(cfg, root_dir=root, include_fast=True, include_slow=True)
        torch.manual_seed(4321)  # the same split and order on every rank
        ds_tr, ds_val, dl, _ = prepare_dataloader_with_split(c, val_split=0.1)
    build_s = time.perf_counter() - t0
    n_frames = sum(len(a) for a, _ in ds_tr.dataset.clips)
    log("C4 corpus: %d clips x %.0f s -> %d frames (fast+slow), %d train windows, built in %.1fs"
        % (args.feed_clips, args.feed_seconds, n_frames, len(ds_tr), build_s))
    it = rank_batches(dl, rank, world) if world > 1 else enumerate(dl)

    def fed_step():
        _, (src, trg) = next(it)
        return step_fn(src.to(dev, non_blocking=True), trg.to(dev, non_blocking=True))

    for _ in range(3):
        fed_step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t1 = time.perf_counter()
    for _ in range(args.feed_steps):
        fed_step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = time.perf_counter() - t1
    if world > 1:
        tt = torch.tensor([el], device=dev)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        el = tt.item()
    B, T = args.batch, args.seq
    return {"value": round(B * T * world * args.feed_steps / el, 1), "unit": "frames/s",
            "ms_per_step": round(el / args.feed_steps * 1e3, 3), "steps": args.feed_steps,
            "corpus": "%d synthetic clips x %.0f s, include_fast + include_slow: %d frames, %d train windows"
                      % (args.feed_clips, args.feed_seconds, n_frames, len(ds_tr)),
            "corpus_build_s": round(build_s, 1),
            "path": "prepare_dataloader_with_split -> DataLoader(batched fetch into pinned host memory, shuffle) "
                    "-> non_blocking H2D -> train step"}


FP32_VECTOR_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md
FP64_VECTOR_PEAK_TFLOPS = 78.6   # half the FP32 vector rate (a wave64 f64 FMA takes 4 cycles on SIMD-32)
# v_mfma_f64_16x16x4_f64 measured alone (tools/micro/mfma_f64_rate.hip,
# profiles/r3_f64_rate_micro.txt); it shares the f64 unit with the vector FMAs
FP64_MFMA_MEASURED_TFLOPS = 49.4


def feature_rooflines(K, audio, n_samp, sr, dev):
    """The feature path's two kernels timed alone on the feature leg's audio (HIP
    events, median of 5), against the resource that bounds each:
    - autocorrelation (the dominant one): 2 * n_fft * (n_lags + 1) f64 FLOP per
      120 Hz frame (direct lag products, as the reference's f64 np.correlate)
      vs the FP64 peak (78.6 TF/s; the kernel runs them on the f64 MFMA, which
      measured 49.4 TF/s alone: frac_of_mfma_measured);
    - fused STFT/mel: 5 n log2 n FLOP per frame (the radix-agnostic FFT count)
      + |X|^2 + mel bands, vs the FP32 vector peak; its algorithmic bytes (audio
      read once, mel power written) vs HBM."""
    import math
    n_fft, hop, n_lags = int(0.01667 * sr), int(0.01667 * sr) // 2, 187
    F = 1 + n_samp // hop

    def med(fn):
        ts = []
        for _ in range(6):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return sorted(ts[1:])[2] * 1e-3
    ac = torch.empty(F, n_lags, dtype=torch.float64, device=dev)
    mel = torch.empty(F, 128, dtype=torch.float32, device=dev)
    t_ac = med(lambda: K.autocorr(audio, n_fft, hop, n_lags, ac, F))
    t_sm = med(lambda: K.stft_mel(audio, n_samp, sr, mel, F))
    ac_flop = 2.0 * n_fft * (n_lags + 1) * F
    sm_flop = (5.0 * n_fft * math.log2(n_fft) + 3 * (n_fft // 2 + 1) + 2 * 2 * (n_fft // 2 + 1)) * F
    sm_bytes = 4.0 * n_samp + 4.0 * 128 * F
    return {"frames_120hz": F,
            "roofline": {"kernel": "autocorr3_kernel (f64 MFMA lag products, the feature path's longest kernel)",
                         "bound": "fp64", "achieved": round(ac_flop / t_ac / 1e12, 2),
                         "peak": FP64_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(ac_flop / t_ac / 1e12 / FP64_VECTOR_PEAK_TFLOPS, 4),
                         "frac_of_mfma_measured": round(ac_flop / t_ac / 1e12 / FP64_MFMA_MEASURED_TFLOPS, 4),
                         "us": round(t_ac * 1e6, 1), "algorithmic_flop": ac_flop},
            "stft_mel": {"kernel": "stft_mel_kernel (fused STFT/mel, mixed-radix f32 FFT in LDS)",
                         "us": round(t_sm * 1e6, 1), "achieved_tflops": round(sm_flop / t_sm / 1e12, 3),
                         "frac_fp32_vector": round(sm_flop / t_sm / 1e12 / FP32_VECTOR_PEAK_TFLOPS, 4),
                         "achieved_gbs": round(sm_bytes / t_sm / 1e9, 1),
                         "frac_hbm": round(sm_bytes / t_sm / 1e9 / PEAK_HBM_GBS, 4)}}


def fwd_parity(cfg, dev, T, windows=2):
    """BASELINE metric's "MSE vs ref" (SURVEY.md 8(d)(i)): forward output of the
    full 228M config (all 8+8 layers) vs the fp32 CPU oracle on the same batch
    and the same seeded weights, in fp32 parity mode (gate <= 1e-3) and in the
    bf16 mode the bench trains in (reported, not gated)."""
    from oracle import model_ref
    from neurosync_trainer_lite_amd.utils.model_utils import build_model
    H = cfg["num_heads"]
    params = model_ref.seeded_params(model_ref.param_shapes(cfg["input_dim"], cfg["hidden_dim"], cfg["n_layers"],
                                                            cfg["output_dim"]), 11)
    g = torch.Generator().manual_seed(12)
    src = torch.randn(windows, T, cfg["input_dim"], generator=g)
    t0 = time.perf_counter()
    with torch.no_grad():
        ref = model_ref.seq2seq_forward(params, src, H).double()
    out = {"windows": windows, "frames": windows * T, "oracle_s": round(time.perf_counter() - t0, 2), "gate": 1e-3}
    modes = [("fp32", False, False), ("bf16", True, False)] + ([("fp8", True, True)] if cfg.get("use_fp8") else [])
    for tag, amp, fp8 in modes:
        c = dict(cfg, use_amp=amp, dropout=0.0, use_fp8=fp8)
        m = build_model(c, dev)
        m.load_state_dict(params, strict=True)
        m.eval()
        with torch.no_grad():
            pred = m(src.to(dev)).double().cpu()
        out["mse_" + tag] = float(((pred - ref) ** 2).mean())
        out["rel_" + tag] = float((pred - ref).norm() / ref.norm())
        del m
        torch.cuda.empty_cache()
    out["pass"] = out["mse_fp32"] <= out["gate"]
    if "mse_fp8" in out:  # C5: the fp8 forward is held to the same gate
        out["pass_fp8"] = out["mse_fp8"] <= out["gate"]
        out["pass"] = out["pass"] and out["pass_fp8"]
    return out


def rank_launch_cmd(args, argv, port):
    """The torch.distributed.run command that starts args.gpus ranks of this
    bench on one node (the form the reference's ≤4-replica loop becomes: one
    process per GPU, /root/reference/train.py:62-78)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(cmd, env, stall_s, limit_s):
    """Run the rank launcher as a child process group: stderr relayed line by
    line, stdout collected.  Killed (the whole group) after stall_s seconds
    without a line on either stream, or after limit_s.  Returns (rc or None if
    killed, stdout lines, last stderr lines, why killed)."""
    import ctypes
    import signal
    import subprocess
    import threading

    def die_with_parent():  # in the child, before exec: SIGTERM when this process dies
        try:
            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
        except OSError:
            pass
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True, preexec_fn=die_with_parent)

    # the ranks run in their own session: a signal that ends this launcher ends them too
    def forward(signum, frame):
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
        raise SystemExit(128 + signum)
    old = {sg: signal.signal(sg, forward) for sg in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)}
    out, tail, last = [], [], [time.monotonic()]

    def pump(src, sink):
        for line in src:
            last[0] = time.monotonic()
            sink(line)

    def err_line(line):
        sys.stderr.write(line)
        sys.stderr.flush()
        tail.append(line.rstrip())
        del tail[:-30]
    ts = [threading.Thread(target=pump, args=(p.stdout, out.append), daemon=True),
          threading.Thread(target=pump, args=(p.stderr, err_line), daemon=True)]
    for t in ts:
        t.start()
    t0, why = time.monotonic(), None
    while p.poll() is None:
        time.sleep(0.5)
        now = time.monotonic()
        if now - last[0] > stall_s:
            why = "no output for %.0f s" % stall_s
        elif now - t0 > limit_s:
            why = "over the %.0f s limit" % limit_s
        if why:
            log("rank launcher %s: stopping its process group" % why)
            for sig, wait in ((signal.SIGTERM, 20), (signal.SIGKILL, 10)):
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    break
                try:
                    p.wait(wait)
                    break
                except subprocess.TimeoutExpired:
                    continue
            break
    for t in ts:
        t.join(5)
    for sg, h in old.items():
        signal.signal(sg, h)
    return (None if why else p.returncode), out, tail, why


def launch_ranks(args, argv):
    """`bench.py --gpus N` (N > 1) without torchrun's environment: start the N
    ranks as a child torch.distributed.run (before this process makes any GPU
    call: torch.cuda.device_count() does not initialise HIP here), relay rank
    0's JSON line with `launch` added, and return the exit code.  With NSTL_DP
    unset the first attempt runs the default exchange (zero1_push, whose
    cross-device copy path first executes on a multi-GPU node); if it fails or
    stalls, a second attempt runs NSTL_DP=zero1 and the line says so
    (config.dp_fallback)."""
    n_dev = torch.cuda.device_count()
    # NSTL_DIST_BACKEND=gloo: a rehearsal with several ranks per GPU (parallel.init_from_env)
    if n_dev < args.gpus and not (n_dev and os.environ.get("NSTL_DIST_BACKEND") == "gloo"):
        log("--gpus %d needs %d GPUs on this node; %d visible" % (args.gpus, args.gpus, n_dev))
        return 2
    modes = [os.environ["NSTL_DP"]] if os.environ.get("NSTL_DP") else ["zero1_push", "zero1"]
    attempts, line = [], None
    for mode in modes:
        cmd = rank_launch_cmd(args, argv, _free_port())
        env = dict(os.environ, NSTL_DP=mode, NSTL_BENCH_SELF_LAUNCH="1", MASTER_ADDR="127.0.0.1")
        log("starting %d ranks (NSTL_DP=%s): %s" % (args.gpus, mode, " ".join(cmd)))
        t0 = time.monotonic()
        rc, out, tail, why = _run_ranks(cmd, env, args.launch_stall_s, args.launch_limit_s)
        js = [ln for ln in out if ln.lstrip().startswith("{")]
        att = {"NSTL_DP": mode, "rc": rc, "s": round(time.monotonic() - t0, 1)}
        if rc == 0 and js:
            attempts.append(att)
            line = json.loads(js[-1])
            break
        att["failure"] = why or ("exit %s" % rc if rc else "no JSON line from rank 0")
        att["stderr_tail"] = tail[-6:]
        attempts.append(att)
        log("attempt NSTL_DP=%s failed: %s" % (mode, att["failure"]))
    if line is None:
        print(json.dumps({"metric": "train frames/sec (audio->blendshape) 228M cfg", "value": None,
                          "n_gpus": args.gpus, "error": "every rank-launch attempt failed",
                          "launch": {"attempts": attempts}}), flush=True)
        return 1
    line["launch"] = {"how": "bench.py --gpus %d started torch.distributed.run --nproc-per-node %d as a child"
                             % (args.gpus, args.gpus), "attempts": attempts}
    if len(attempts) > 1:
        line["config"]["dp_fallback"] = "NSTL_DP=%s attempt failed (%s); measured with NSTL_DP=%s" % (
            attempts[0]["NSTL_DP"], attempts[0]["failure"], attempts[-1]["NSTL_DP"])
    print(json.dumps(line), flush=True)
    return 0


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the forward-MSE-vs-oracle field")
    ap.add_argument("--gemm-sample-steps", type=int, default=1,
                    help="timed steps (the last ones) whose GEMM launches carry HIP timing events")
    ap.add_argument("--feature-steps", type=int, default=10,
                    help="steps of the feature-inclusive variant (raw audio -> GPU features -> step); 0 = skip")
    ap.add_argument("--feed-steps", type=int, default=20,
                    help="steps of the C4 data-feed variant (synthetic corpus with fast+slow augmentation through "
                         "the DataLoader with pinned non_blocking H2D); 0 = skip")
    ap.add_argument("--feed-clips", type=int, default=16)
    ap.add_argument("--feed-seconds", type=float, default=60.0)
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the rocprofv3 counter passes that measure the GEMM family's HBM traffic")
    ap.add_argument("--fp8", action="store_true",
                    help="BASELINE config C5: q/k/v + FFN forward GEMMs on e4m3 operands (row-wise scales); "
                         "C5 also doubles the clip length: --seq 256 --batch 64")
    ap.add_argument("--fp8-bwd", action="store_true",
                    help="with --fp8: every FFN linear2 input-gradient GEMM on e4m3 operands too")
    ap.add_argument("--launch-stall-s", type=float, default=300.0,
                    help="--gpus N self-launch: an attempt with no output line for this long is stopped")
    ap.add_argument("--launch-limit-s", type=float, default=1500.0,
                    help="--gpus N self-launch: an attempt running longer than this is stopped")
    args = ap.parse_args(argv)

    env_world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if env_world == 0 and args.gpus > 1:
        # N ranks wanted and not started by torchrun: start them (no GPU call here)
        sys.exit(launch_ranks(args, sys.argv[1:] if argv is None else argv))
    if env_world and env_world != args.gpus:
        raise SystemExit("bench.py --gpus %d, but this rank was started in a world of %d (WORLD_SIZE): pass "
                         "--gpus %d or start %d ranks" % (args.gpus, env_world, env_world, args.gpus))

    from neurosync_trainer_lite_amd import _hip as K
    from neurosync_trainer_lite_amd import parallel
    from neurosync_trainer_lite_amd.config import training_config
    from neurosync_trainer_lite_amd.utils.model_utils import build_model, prepare_training_components
    from neurosync_trainer_lite_amd.utils.training_utils import gradient_exchange

    # PMC traffic passes first: child processes, started before this one touches the GPU
    traffic, traffic_src, mfma_busy = None, "skipped (--no-traffic or n>1)", None
    counters = {}
    if int(os.environ.get("WORLD_SIZE", "1")) == 1 and not args.no_traffic:
        counters = measure_gemm_counters(args)
        traffic, traffic_src, mfma_busy = counters["traffic"], counters["note"], counters["mfma_busy"]
    rank, world, local = parallel.init_from_env()
    if world != args.gpus:
        raise SystemExit("bench.py --gpus %d ran in a world of %d" % (args.gpus, world))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cfg = dict(training_config)
    B, T = args.batch, args.seq
    cfg.update(micro_batch_size=T, frame_size=T, batch_size=B, use_fp8=args.fp8, fp8_backward=args.fp8_bwd)
    torch.manual_seed(1234)  # identical init on every rank
    model = build_model(cfg, dev)
    model.train()
    crit, opt, sched = prepare_training_components(cfg, model)
    eng = model.engine()
    if world > 1:
        # sharded optimizer (ZeRO-1; NSTL_DP=allreduce: bucketed all-reduce during backward)
        from neurosync_trainer_lite_amd.utils.training_utils import attach_data_parallel
        attach_data_parallel(model, opt, world)
    W = sum(p.numel() for n, p in model.named_parameters() if n.endswith("weight") and p.dim() == 2)

    g = torch.Generator(device=dev).manual_seed(100 + rank)
    src = torch.randn(B, T, cfg["input_dim"], device=dev, generator=g)
    trg = torch.randn(B, T, cfg["output_dim"], device=dev, generator=g) * 20

    # as train_one_epoch sets it: nothing writes the gradients between backward
    # and step, so the clip norm may come from the weight-gradient epilogues'
    # partials.
    opt.trust_backward_norm = world == 1
    # as train_one_epoch: the next use of the parameters is the next forward, so the
    # update MAY run under it -- only with NSTL_ADAM_OVERLAP=1 (FusedAdam: opt-in)
    opt.overlap_next_forward = True

    def step(x=src, y=trg):
        opt.zero_grad()
        loss = crit(model(x), y)
        loss.backward()
        opt.step(max_norm=2.0)
        return loss

    t_w = time.perf_counter()
    for i in range(args.warmup):
        step()
        torch.cuda.synchronize()
        log("warm-up step %d done at %.2fs" % (i, time.perf_counter() - t_w))

    # live per-launch timing of the dominant kernel (GEMM) inside the timed region
    # (events and stream wrappers made before the clock starts).  Each timing
    # event waits for the kernel before it to drain, so a sampled step runs
    # ~1-2 ms slower (tools/gap_check.py on a kernel trace: 155-319 gaps of
    # 5-15 us); one sampled step keeps that out of the other timed steps.
    gemm_events = []
    real_gemm = K.gemm
    ev_pool = [torch.cuda.Event(enable_timing=True) for _ in range(1200 * max(1, args.gemm_sample_steps))]
    streams = {}

    def stream_of(handle):
        # the stream a GEMM is launched on (weight-gradient GEMMs run on a side stream)
        if not handle:
            return torch.cuda.current_stream()
        st = streams.get(handle)
        if st is None:
            st = streams[handle] = torch.cuda.ExternalStream(handle)
        return st

    def take_events():
        if len(ev_pool) >= 2:
            return ev_pool.pop(), ev_pool.pop()
        return torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def launched_family():
        # which kernel the last nstl_gemm call ran (launch counters, sampled steps only)
        c = K.kernel_counts()
        K.kernel_counts_reset()
        if c["gemm4"]:
            return "gemm4"
        if c["gemm_ring"] or c["gemm_group"]:
            return "ring"
        return "gemm128" if c["gemm128"] else "other"

    def timed_gemm(A, B_, C, M, N, Kd, **kw):
        if not sample[0]:
            real_gemm(A, B_, C, M, N, Kd, **kw)
            return
        st = stream_of(kw.get("stream"))
        e0, e1 = take_events()
        K.kernel_counts_reset()
        e0.record(st)
        real_gemm(A, B_, C, M, N, Kd, **kw)
        e1.record(st)
        ebytes = A.element_size()
        cbytes = C.element_size()
        gemm_events.append((e0, e1, 2.0 * M * N * Kd, (M * Kd + N * Kd) * ebytes + M * N * cbytes, ebytes == 1, False,
                            launched_family()))

    # Timing events around every launch cost ~1.7 ms per step (228M), so they are
    # recorded in the last `--gemm-sample-steps` timed steps only.
    sample = [False]
    real_grouped = K.gemm_grouped

    def timed_grouped(problems, stream=None):
        if not sample[0]:
            real_grouped(problems, stream=stream)
            return
        st = stream_of(stream)
        e0, e1 = take_events()
        K.kernel_counts_reset()
        e0.record(st)
        real_grouped(problems, stream=stream)
        e1.record(st)
        fl = sum(2.0 * M * N * Kd for _, _, _, M, N, Kd, _ in problems)
        by = sum((M * Kd + N * Kd) * A.element_size() + M * N * C.element_size() for A, _, C, M, N, Kd, _ in problems)
        fam = launched_family()
        # the weight gradients (f32 out) vs the decoder's grouped cross k|v + RoPE projections (bf16 out)
        dw = all(C.dtype == torch.float32 for _, _, C, _, _, _, _ in problems)
        gemm_events.append((e0, e1, fl, by, False, dw, "gemm4_grouped_dw" if fam == "gemm4" and dw else fam))

    K.gemm = timed_gemm
    K.gemm_grouped = timed_grouped
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        sample[0] = i >= args.steps - args.gemm_sample_steps
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    K.gemm = real_gemm
    K.gemm_grouped = real_grouped
    rank_ms = None
    if world > 1:
        tt = torch.tensor([elapsed], device=dev)
        per = [torch.zeros(1, device=dev) for _ in range(world)]
        torch.distributed.all_gather(per, tt)
        rank_ms = [round(float(x) / args.steps * 1e3, 3) for x in per]
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        elapsed = tt.item()
    log("timed %d steps in %.3fs" % (args.steps, elapsed))
    loss_v = loss.item()
    if not (loss_v == loss_v):
        raise RuntimeError("non-finite loss %r" % loss_v)

    # bf16 launches -> `roofline` (vs the bf16 peak); fp8 launches (--fp8) -> `roofline_fp8`
    ev16 = [e for e in gemm_events if not e[4]]
    ev8 = [e for e in gemm_events if e[4]]
    all_ms = sum(a.elapsed_time(b) for a, b, _, _, _, _, _ in gemm_events)
    gemm_ms = sum(a.elapsed_time(b) for a, b, _, _, _, _, _ in ev16)
    gemm_flops = sum(f for _, _, f, _, _, _, _ in ev16)
    gemm_alg_bytes = sum(x for _, _, _, x, _, _, _ in ev16) / max(1, len(ev16))
    n_launch = len(ev16)
    fp8_roof = None
    if ev8:
        ms8 = sum(a.elapsed_time(b) for a, b, _, _, _, _, _ in ev8)
        tf8 = sum(f for _, _, f, _, _, _, _ in ev8) / (ms8 * 1e-3) / 1e12
        fp8_roof = {"bound": "mfma", "kernel": "gemm256f8_kernel (e4m3 operands, row scales; which GEMMs: config.fp8_scope)",
                    "achieved": round(tf8, 1), "peak": FP8_DENSE_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(tf8 / FP8_DENSE_PEAK_TFLOPS, 4), "launches": len(ev8),
                    "avg_launch_us": round(ms8 * 1e3 / len(ev8), 2),
                    "algorithmic_bytes_per_launch": round(sum(x for _, _, _, x, _, _, _ in ev8) / len(ev8)),
                    "share_of_step": round(ms8 / (max(1, min(args.steps, args.gemm_sample_steps)) * elapsed / args.steps * 1e3), 3)}
    n_sampled = max(1, min(args.steps, args.gemm_sample_steps))
    # the largest single kernel by time: the grouped weight-gradient launches
    # (gemm4_kernel, grouped NN form), the kernel round 1's verdict priced on its own
    evg = [e for e in ev16 if e[5]]
    dom_roof = None
    if evg:
        msg = sum(a.elapsed_time(b) for a, b, _, _, _, _, _ in evg)
        tfg = sum(f for _, _, f, _, _, _, _ in evg) / (msg * 1e-3) / 1e12
        dom_roof = {"bound": "mfma", "kernel": "gemm4_kernel<false, false, EM_F32, grouped> (grouped weight gradients, "
                                               "f32 into the gradient arena; decoder layer = 1 launch, 4 encoder "
                                               "layers = 1)",
                    "achieved": round(tfg, 1), "peak": BF16_DENSE_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(tfg / BF16_DENSE_PEAK_TFLOPS, 4), "launches": len(evg),
                    "avg_launch_us": round(msg * 1e3 / len(evg), 2),
                    "algorithmic_bytes_per_launch": round(sum(x for _, _, _, x, _, _, _ in evg) / len(evg)),
                    "share_of_step": round(msg / (n_sampled * elapsed / args.steps * 1e3), 3)}
    achieved_tf = gemm_flops / (gemm_ms * 1e-3) / 1e12 if gemm_ms > 0 else 0.0
    # the same per kernel family (which kernel each launch ran: launch counters)
    by_family = {}
    for fam in ("gemm4", "gemm4_grouped_dw", "ring", "gemm128"):
        ev = [e for e in ev16 if e[6] == fam]
        if not ev:
            continue
        ms_f = sum(a.elapsed_time(b) for a, b, _, _, _, _, _ in ev)
        tf_f = sum(f for _, _, f, _, _, _, _ in ev) / (ms_f * 1e-3) / 1e12
        by_family[fam] = {"launches": len(ev), "achieved": round(tf_f, 1),
                          "frac": round(tf_f / BF16_DENSE_PEAK_TFLOPS, 4),
                          "avg_launch_us": round(ms_f * 1e3 / len(ev), 2),
                          "algorithmic_bytes_per_launch": round(sum(x for _, _, _, x, _, _, _ in ev) / len(ev)),
                          "share_of_step": round(ms_f / (n_sampled * elapsed / args.steps * 1e3), 3)}
    ms_step = elapsed / args.steps * 1e3
    frames = B * T * world * args.steps
    value = frames / elapsed
    step_tf = frames_flops(W, T, cfg["hidden_dim"]) * B * T * world / (elapsed / args.steps) / 1e12 / world

    # feature-inclusive variant (BASELINE C2's on-GPU STFT/mel path): per step,
    # raw 88.2 kHz audio for the step's B*T frames -> nstl_features -> windows
    feat = None
    if args.feature_steps > 0:
        from neurosync_trainer_lite_amd.utils.audio.extraction.extract_features import extract_audio_features_device
        sr = cfg["sr"]
        n_samp = int(B * T / 60.0 * sr) + 1470
        tt = torch.arange(n_samp, device=dev, dtype=torch.float32) / sr
        gen = torch.Generator(device=dev).manual_seed(7 + rank)
        audio = (0.6 * torch.sin(2 * 3.14159265 * 180.0 * tt) * (0.55 + 0.45 * torch.sin(2 * 3.14159265 * 4.0 * tt))
                 + 0.01 * torch.randn(n_samp, device=dev, generator=gen))
        audio = audio / audio.abs().max()

        def feat_step():
            f = extract_audio_features_device(audio, sr, device=dev)
            src_f = f[:B * T].view(B, T, -1)
            opt.zero_grad()
            loss_f = crit(model(src_f), trg)
            loss_f.backward()
            opt.step(max_norm=2.0)
            return loss_f

        feat_step()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        t1 = time.perf_counter()
        for _ in range(args.feature_steps):
            feat_step()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        el_f = time.perf_counter() - t1
        if world > 1:
            tt_ = torch.tensor([el_f], device=dev)
            torch.distributed.all_reduce(tt_, op=torch.distributed.ReduceOp.MAX)
            el_f = tt_.item()
        # the same work as a two-stage pipeline: step i+1's features are extracted on
        # a side stream while step i trains (a prefetching loader's schedule); all
        # feature_steps extractions run inside the timed region
        side = torch.cuda.Stream(dev)
        main = torch.cuda.current_stream(dev)

        def extract_side():
            with torch.cuda.stream(side):
                f = extract_audio_features_device(audio, sr, device=dev)
                ev = torch.cuda.Event()
                ev.record(side)
            return f, ev

        def pipelined(n):
            f, ev = extract_side()
            for i in range(n):
                main.wait_event(ev)
                f.record_stream(main)
                nxt = extract_side() if i + 1 < n else None
                src_f = f[:B * T].view(B, T, -1)
                opt.zero_grad()
                loss_p = crit(model(src_f), trg)
                loss_p.backward()
                opt.step(max_norm=2.0)
                if nxt is not None:
                    f, ev = nxt
        pipelined(2)
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        t2 = time.perf_counter()
        pipelined(args.feature_steps)
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        el_p = time.perf_counter() - t2
        if world > 1:
            tt_ = torch.tensor([el_p], device=dev)
            torch.distributed.all_reduce(tt_, op=torch.distributed.ReduceOp.MAX)
            el_p = tt_.item()
        # extraction alone: 5 back-to-back calls (one call alone would time the
        # host's launches into an idle stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            extract_audio_features_device(audio, sr, device=dev)
        e1.record()
        torch.cuda.synchronize()
        feat = {"value": round(B * T * world * args.feature_steps / el_f, 1), "unit": "frames/s",
                "ms_per_step": round(el_f / args.feature_steps * 1e3, 3), "steps": args.feature_steps,
                "feature_ms_per_step": round(e0.elapsed_time(e1) / 5, 3),
                "pipelined_value": round(B * T * world * args.feature_steps / el_p, 1),
                "pipelined_ms_per_step": round(el_p / args.feature_steps * 1e3, 3),
                "pipelined": "step i+1's extraction on a side stream under step i (same extractions, same steps)",
                "workload": "per step: %.1f s of synthetic 88.2 kHz audio per GPU -> GPU MFCC(+d,dd)+autocorr "
                            "features [%d frames x 256] -> the same train step" % (n_samp / sr, B * T)}
        feat.update(feature_rooflines(K, audio, n_samp, sr, dev))
        feat["roofline"]["share_of_features"] = round(feat["roofline"]["us"] * 1e-3 / feat["feature_ms_per_step"], 3)
        feat["vs_resident"] = round(feat["value"] / value, 4)
        feat["pipelined_vs_resident"] = round(feat["pipelined_value"] / value, 4)

    feed = None
    if args.feed_steps > 0:
        feed = data_feed(cfg, args, step, dev, rank, world)
        feed["vs_resident"] = round(feed["value"] / value, 4)

    if rank == 0:
        out = {
            "metric": "train frames/sec (audio->blendshape) 228M cfg",
            "value": round(value, 1),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (seeded features [B,T,256] + targets [B,T,61], resident in HBM)",
            "config": {"workload": "228M Seq2Seq train step (L8/H16/D1024, dropout 0.3, clip+Adam)",
                       "model": "NeuroSync Seq2Seq 228M", "global_batch": B * world, "seq_len": T,
                       "frames_per_step": B * T * world, "parallelism": "dp%d" % world,
                       "gradient_exchange": gradient_exchange(model, opt),
                       "dp_fallback": (None if world == 1 else opt.dp_fallback or False)},
            "roofline": {"bound": "mfma", "kernel": "nstl GEMM family, all hand-written: gemm4_kernel (4-wave persistent "
                                                    "256^2: every full-tile forward / dX / grouped dW), gemm256r_kernel "
                                                    "(8-wave ring: f32 beta-1 dX, the memory gradient), gemm_kernel "
                                                    "(128^2: small shapes); every launch of the last %d timed steps"
                                                    % n_sampled,
                         "achieved": round(achieved_tf, 1), "peak": BF16_DENSE_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved_tf / BF16_DENSE_PEAK_TFLOPS, 4), "traffic": traffic,
                         "traffic_unit": "HBM bytes per launch (PMC: 2*FETCH_SIZE + WRITE_SIZE)",
                         "traffic_vs_algorithmic": (round(traffic / gemm_alg_bytes, 3) if traffic and gemm_alg_bytes
                                                    else None),
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": round(gemm_alg_bytes),
                         "launches": n_launch, "avg_launch_us": round(gemm_ms * 1e3 / max(1, n_launch), 2),
                         "gemm_share_of_step": round(all_ms / (n_sampled * ms_step), 3)},
            "step_tflops_per_gpu": round(step_tf, 1),
            "step_mfma_frac": round(step_tf / BF16_DENSE_PEAK_TFLOPS, 4),
            "final_loss": round(loss_v, 4),
        }
        if world > 1:
            out["dist"] = {"backend": torch.distributed.get_backend(), "world_size": torch.distributed.get_world_size(),
                           "launch": ("bench.py self-launch (torch.distributed.run child)"
                                      if os.environ.get("NSTL_BENCH_SELF_LAUNCH") == "1" else "external torchrun"),
                           "rank_ms_per_step": rank_ms,
                           "rank_spread_pct": round((max(rank_ms) / min(rank_ms) - 1) * 100, 2),
                           "exchange_check": opt.dp_check}
        fam_traffic = counters.get("traffic_by_family") or {}
        for fam, d in by_family.items():
            t = fam_traffic.get(fam)
            if t:
                d["traffic"] = t["traffic"]
                d["traffic_vs_algorithmic"] = round(t["traffic"] / d["algorithmic_bytes_per_launch"], 3)
            if mfma_busy is not None and mfma_busy["by_family"].get(fam):
                d["mfma_busy"] = mfma_busy["by_family"][fam]
        out["roofline"]["by_family"] = by_family
        if mfma_busy is not None:
            out["roofline"]["mfma_busy"] = mfma_busy["gemm_family"]
        if dom_roof is not None:
            if mfma_busy is not None:
                dom_roof["mfma_busy"] = mfma_busy["grouped_dw"]
                dom_roof["mfma_busy_source"] = mfma_busy["source"]
            out["roofline_dominant"] = dom_roof
        if fp8_roof is not None:
            scope = eng.fp8_scope_desc() if hasattr(eng, "fp8_scope_desc") else None
            fp8_roof["scope"] = scope
            out["roofline_fp8"] = fp8_roof
            out["dtype"] = "bf16 + e4m3 (%s; row-wise scales)" % (scope["summary"] if scope else "fp8 GEMMs")
            out["config"]["workload"] = ("C5: 228M Seq2Seq train step (L8/H16/D1024, dropout 0.3, clip+Adam), "
                                         "fp8 %s, T=%d" % (scope["summary"] if scope else "GEMMs", T))
            out["config"]["fp8_scope"] = scope
        if feat is not None:
            out["feature_inclusive"] = feat
        if feed is not None:
            out["data_feed"] = feed
        if world == 1 and not args.no_parity:
            out["parity"] = fwd_parity(cfg, dev, T)
            log("parity: %s" % out["parity"])
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cfg, T)
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
