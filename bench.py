"""Benchmark: Flow.log_prob samples/s (+ NLL) on the BASELINE.json headline
config — 4D rolling spline coupling flow, K=16 knots, 4 couplings, hidden
(128, 128), Normal latent, batch 2^20 per GPU — through the fused HIP kernel.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2]

One process per GPU, no torch: ``--gpus N`` (N>1) spawns N fresh ranks
itself (zenflow_amd.launch.spawn) unless the env already holds a launch
(``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N``,
the driver's form).  Ranks meet in a file rendezvous (RCCL unique id,
barriers, max-over-ranks timing).  A step is one log_prob pass over the
rank's resident 2^20-row shard (zenflow_amd.dist.DataParallelLogProb): the
fused kernel (ShiftBounds -> 4x[MLP on MFMA + RQ spline] -> Normal latent ->
flow.py:47 -> per-block fp64 NLL partials), the fixed-order NLL reduce and,
for N>1, the RCCL all-reduce of the NLL (overlapped on a communication
stream).  Rank 0 prints one JSON line."""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

PEAK_FP32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense fp32 MFMA (no xf32 on gfx950)
PEAK_BF16_MFMA_TFLOPS = 2516.6  # dense bf16 MFMA: 256 CU x 4 SIMD x 1024 flop/clk x 2.4 GHz
# fp32-accurate GEMM by the three-term bf16 split: 6 bf16 products per fp32 product
PEAK_BF16X3_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 6
# two-term fp16 split of power-of-two-scaled operands: 3 fp16 products (fp16 dense = bf16 dense rate)
PEAK_F16X2_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 3
SPLIT_PEAKS = {
    "bf16x3": (PEAK_BF16X3_TFLOPS, "bf16 dense MFMA peak / 6 (three-term bf16 split, fp32-equivalent flops)"),
    "f16x2": (PEAK_F16X2_TFLOPS, "fp16 dense MFMA peak / 3 (two-term fp16 split, fp32-equivalent flops)"),
}
PEAK_HBM_GBS = 8000.0
PEAK_CLOCK_GHZ = 2.4  # the clock every MFMA peak above assumes

WORKLOADS = {
    # name: (D, C, K, layers, couplings, latent, mode)
    # cfg1: two_moons through the drop-in API (host arrays in and out, the
    # FLAX-style apply of examples/two_moons.ipynb), batch 4096
    "cfg1": (2, 0, 8, (128, 128), 2, "beta", "apply"),
    "cfg2": (4, 0, 16, (128, 128), 4, "normal", "log_prob"),
    "cfg3": (4, 0, 16, (128, 128), 4, "normal", "inverse"),
    "cfg3s": (4, 0, 16, (128, 128), 4, "normal", "sample"),  # Flow.sample, latent drawn on device
    "cfg4": (2, 2, 16, (128, 128), 2, "beta", "log_prob"),
    "cfg5": (16, 0, 32, (256, 256), 8, "normal", "log_prob"),
    # reference defaults at dim 8 (rolling_spline_coupling(8): 8 couplings,
    # knots 16, layers (128, 128)), and K = 32 at hidden 128
    "d8": (8, 0, 16, (128, 128), 8, "normal", "log_prob"),
    "d4k32": (4, 0, 32, (128, 128), 4, "normal", "log_prob"),
    # cfg2 with NeuralSplineCoupling(act=...) other than swish (bijectors.py:319)
    "cfg2relu": (4, 0, 16, (128, 128), 4, "normal", "log_prob", "relu"),
    "cfg2gelu": (4, 0, 16, (128, 128), 4, "normal", "log_prob", "gelu"),
    "cfg2sigmoid": (4, 0, 16, (128, 128), 4, "normal", "log_prob", "sigmoid"),
    "cfg2softplus": (4, 0, 16, (128, 128), 4, "normal", "log_prob", "softplus"),
}


def workload(name):
    """(D, C, K, layers, couplings, latent, mode, act) of a bench workload."""
    w = WORKLOADS[name]
    return tuple(w[:7]) + ((w[7] if len(w) > 7 else "swish"),)


def build_model(name):
    import zenflow_amd as zf
    from zenflow_amd import bijectors as bi
    from zenflow_amd import distributions as dist

    D, C, K, layers, L, latent, mode, act = workload(name)
    bij = [bi.ShiftBounds(margin=0.1)]
    for _ in range(L - 1):
        bij += [bi.NeuralSplineCoupling(knots=K, layers=layers, act=act), bi.Roll()]
    bij.append(bi.NeuralSplineCoupling(knots=K, layers=layers, act=act))
    lat = dist.Normal() if latent == "normal" else dist.Beta()
    return zf.Flow(bi.Chain(bij), latent=lat)


def flops_per_sample(name):
    """2 * MACs of the conditioner MLPs: 2*L*[(dc+C)H + H*H + H*dt*S]."""
    D, C, K, layers, L, _, _, _ = workload(name)
    dt, dc = D // 2, D - D // 2
    widths = [dc + C] + list(layers) + [dt * (3 * K - 1)]
    return 2 * L * sum(a * b for a, b in zip(widths[:-1], widths[1:]))


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_rate(model_spec, variables, x, c, threads, budget_s, chunk, reps, keep_outs):
    from oracle import zf_oracle as O
    from threadpoolctl import threadpool_limits

    N = x.shape[0]
    with threadpool_limits(limits=threads):
        t0 = time.perf_counter()
        O.flow_log_prob(model_spec, variables, x[:chunk], None if c is None else c[:chunk])  # warm-up
        rate = min(chunk, N) / (time.perf_counter() - t0)
        rows = int(min(N, max(chunk, rate * budget_s / (reps + 1))))
        rows = max(min(chunk, N), rows // chunk * chunk)
        rates, outs = [], []
        for rep in range(reps):
            t0 = time.perf_counter()
            for lo in range(0, rows, chunk):
                xs = x[lo : min(rows, lo + chunk)]
                cs = None if c is None else c[lo : lo + xs.shape[0]]
                lp, _ = O.flow_log_prob(model_spec, variables, xs, cs)
                if rep == 0 and keep_outs:
                    outs.append((lo, lp))
            rates.append(rows / (time.perf_counter() - t0))
    return float(np.median(rates)), rows, rates, outs


def cpu_baseline(model_spec, variables, x, c, budget_s=24.0, chunk=1 << 16, reps=5):
    """The oracle (NumPy fp32 restatement of the reference's array graph) on
    the host cores, timed twice: with BLAS threads = every
    CPU this process may use (os.sched_getaffinity), and capped at the
    OMP_NUM_THREADS the GPU box grants one GPU (16); ``value`` is the faster
    of the two, ``cores`` its thread count.  2^16-row chunks; one warm-up
    chunk, then ``reps`` timed passes over a bounded sample, median."""
    host = len(os.sched_getaffinity(0))
    capped = min(host, int(os.environ.get("OMP_NUM_THREADS", host)))
    runs = {}
    outs = None
    for threads in sorted({host, capped}):
        r, rows, rates, o = _cpu_rate(model_spec, variables, x, c, threads, budget_s / 2, chunk, reps, outs is None)
        runs[threads] = (r, rows, rates)
        if outs is None:
            outs = o
    best = max(runs, key=lambda t: runs[t][0])
    r, rows, rates = runs[best]
    return {
        "value": r,
        "unit": "samples/s",
        "cores": int(best),
        "kind": "port",
        "sample": f"{rows} rows of the same batch in {chunk}-row chunks, median of {reps} passes after a "
                  f"warm-up chunk; NumPy fp32 oracle (JAX-CPU reference not importable); BLAS threads={best} "
                  f"(the faster of all {host} affinity CPUs and the OMP_NUM_THREADS={capped} cap)",
        "by_threads": {str(t): {"samples_per_s": v[0], "rows": v[1]} for t, v in runs.items()},
        "host_cpus": host,
        "cpu_model": cpu_model(),
        "pass_rates": rates,
    }, outs


def spline_kernel_roofline(M, N, K, steps):
    """K1 (utils.rational_quadratic_spline_forward boundary) at one coupling's
    shapes: x (M, N), dx/dy (M, N, K), slope (M, N, K-1) resident in HBM.
    Algorithmic bytes = M*(N*(4*3K + 4) + 4); HBM-bound."""
    from zenflow_amd import _lib as L
    from zenflow_amd._lib import DeviceArray, Event

    lib = L.load_library()
    rng = np.random.default_rng(7)
    x = DeviceArray.from_numpy(rng.uniform(-0.05, 1.05, (M, N)).astype(np.float32))
    dx = DeviceArray.from_numpy(rng.standard_normal((M, N, K)).astype(np.float32))
    dy = DeviceArray.from_numpy(rng.standard_normal((M, N, K)).astype(np.float32))
    sl = DeviceArray.from_numpy(rng.standard_normal((M, N, K - 1)).astype(np.float32))
    # utils.normalize_spline_params on copies of the raw logits (in place;
    # repeated runs stay finite), then once on the K1 inputs themselves
    cdx, cdy, csl = DeviceArray(dx.shape), DeviceArray(dy.shape), DeviceArray(sl.shape)
    cdx.copy_from(dx)
    cdy.copy_from(dy)
    csl.copy_from(sl)
    L.check(lib.zf_normalize_spline_params(dx.ptr, dy.ptr, sl.ptr, M * N, K, L.stream()), "normalize")
    y = DeviceArray((M, N))
    ld = DeviceArray((M,))
    xi = DeviceArray((M, N))
    out = {"check": None}
    for tag in ("forward", "inverse", "normalize"):
        def run():
            if tag == "normalize":
                L.check(lib.zf_normalize_spline_params(cdx.ptr, cdy.ptr, csl.ptr, M * N, K, L.stream()), "normalize")
            elif tag == "forward":
                L.check(lib.zf_rqs_forward(x.ptr, dx.ptr, dy.ptr, sl.ptr, y.ptr, ld.ptr, M, N, K, L.stream()), "rqs")
            else:
                L.check(lib.zf_rqs_inverse(y.ptr, dx.ptr, dy.ptr, sl.ptr, xi.ptr, M, N, K, L.stream()), "rqs")
        for _ in range(3):
            run()
        evs = [(Event(), Event()) for _ in range(steps)]
        for a, b in evs:
            a.record()
            run()
            b.record()
        L.synchronize()
        t = float(np.mean([a.elapsed_ms(b) for a, b in evs])) * 1e-3
        if tag == "normalize":  # read + write dx, dy, slope
            nbytes = 2 * M * N * 4 * (3 * K - 1)
            kname = "normalize_vec_kernel"
        else:
            nbytes = M * (N * (4 * 3 * K + 4) + (4 if tag == "forward" else 0))
            kname = ("rqs_kernel_pair" if K == 32 and N <= 128 and not os.environ.get("ZF_K1_ONE_LANE")
                     else "rqs_kernel_direct" if K in (4, 8, 16, 32) else "rqs_kernel")
        gbs = nbytes / t / 1e9
        out[tag] = {"kernel": kname, "shape": [M, N, K], "us": t * 1e6, "alg_bytes": nbytes,
                    "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS}
    # outputs of the timed launches at the timed shape vs the oracle, on a
    # strided row sample (the full-shape test is tests/test_gpu_rqs.py)
    from oracle import zf_oracle as O

    rows = sample_rows(M, 8192)
    hx, hdx, hdy, hsl = x.numpy()[rows], dx.numpy()[rows], dy.numpy()[rows], sl.numpy()[rows]
    yr, ldr = O.rqs_forward(hx, hdx, hdy, hsl)
    xr = O.rqs_inverse(y.numpy()[rows], hdx, hdy, hsl)
    gy, gld, gxi = y.numpy()[rows], ld.numpy()[rows], xi.numpy()[rows]

    def err(a, b):
        f = np.isfinite(a) & np.isfinite(b)
        return {"max_abs_err": float(np.abs(a[f] - b[f]).max()) if f.any() else None,
                "finiteness_mismatches": int((np.isfinite(a) != np.isfinite(b)).sum())}

    out["check"] = {"rows": int(len(rows)), "y": err(gy, yr), "log_det": err(gld, ldr), "inverse": err(gxi, xr)}
    return out


def oracle_spec(name):
    D, C, K, layers, L, latent, _, act = workload(name)
    bij = [{"type": "shift_bounds", "margin": 0.1, "bounds": ()}]
    for _ in range(L - 1):
        bij += [{"type": "nsc", "knots": K, "layers": list(layers), "act": act}, {"type": "roll", "shift": 1}]
    bij.append({"type": "nsc", "knots": K, "layers": list(layers), "act": act})
    return {"bijector": {"type": "chain", "bijectors": bij}, "latent": {"type": latent}}


def load_pmc(kernel_prefix):
    """The committed PMC summaries of the headline kernel: HBM bytes per
    launch (profiles/pmc_traffic.json, scripts/summarize_profiles.py over
    FETCH_SIZE / WRITE_SIZE passes of this bench) and the matrix / vector
    pipe fractions (profiles/x3_pipe_counters.json, scripts/summarize_stall.py
    over the SQ passes of scripts/pmc_stall.sh), or {}."""
    out = {}
    for fname in ("pmc_traffic.json", "x3_pipe_counters.json"):
        try:
            out.update(json.loads((ROOT / "profiles" / fname).read_text()).get(kernel_prefix, {}))
        except (OSError, ValueError):
            pass
    return out


def make_workload(name, N, rank=0):
    """Model, variables and a synthetic input shard of one bench workload:
    random-init weights of the named architecture (flax default
    initialisers), then one train-mode pass over a separate 2^16 batch to set
    the ShiftBounds min/max and BatchNorm running statistics."""
    from zenflow_amd.random import PRNGKey

    D, C, K, layers, nL, latent, mode, act = workload(name)
    flow = build_model(name)
    xinit = np.random.default_rng(3).standard_normal((1 << 16, D)).astype(np.float32)
    cinit = np.random.default_rng(4).standard_normal((1 << 16, C)).astype(np.float32) if C else None
    variables = flow.init(PRNGKey(1), xinit[:1], None if cinit is None else cinit[:1])
    _, upd = flow.apply(variables, xinit, cinit, train=True, mutable=["batch_stats"])
    variables = {"params": variables["params"], "batch_stats": upd["batch_stats"]}
    rng = np.random.default_rng(1000 + rank)
    x = rng.standard_normal((N, D)).astype(np.float32)  # synthetic Gaussian shard
    if mode == "inverse":
        x = (0.5 + 0.1 * rng.standard_normal((N, D))).astype(np.float32)
    c = rng.standard_normal((N, C)).astype(np.float32) if C else None
    return flow, variables, x, c


def run_config(name, N, world):
    """The `config` object of the bench line: the workload, rows per GPU and
    the global batch (weak scaling: N rows per rank)."""
    D, C, K, layers, nL, latent, mode, act = workload(name)
    return {
        "workload": f"{name}: Flow(rolling_spline_coupling({D}, knots={K}, layers={list(layers)}"
                    + ("" if act == "swish" else f", act={act}") + ")"
                    f"{' x' + str(nL) + ' couplings' if nL != D else ''}, latent={latent}).{mode}, "
                    f"{N} rows per GPU, resident in HBM",
        "rows_per_gpu": N,
        "global_batch": N * world,
        "parallelism": f"dp{world} (batch shards, RCCL all-reduce of the fp64 NLL)",
    }


def sample_rows(N, n=4096):
    """A strided sample of n rows spanning the whole batch."""
    return np.arange(0, N, max(1, N // n))[:n]


def logprob_parity(spec, variables, x, c, lp, rows):
    """GPU log_prob on sampled rows vs the oracle (tests/test_gpu_flow.py's
    bars): north_star's unwidened strict error against the fp32 oracle on all
    rows and on the well-conditioned ones (row sensitivity <= 2.5e-6), the
    GPU's and the fp32 oracle's errors against fp64, the conditioned
    tolerance, and the NLL of the same rows (train.py:75-78) from both."""
    from oracle import zf_oracle as O
    from zenflow_amd.dist import nll_from_sum

    xs, cs = x[rows], (None if c is None else c[rows])
    g = lp[rows].astype(np.float64)
    r32, _ = O.flow_log_prob(spec, variables, xs, cs)
    r64, _ = O.flow_log_prob(spec, variables, xs, cs, dtype=np.float64)
    sens = O.row_sensitivity(spec, variables, xs, cs)
    r32 = r32.astype(np.float64)
    fin = np.isfinite(r32) & np.isfinite(g)
    mism = int((np.isfinite(r32) != np.isfinite(g)).sum())
    e_all = np.abs(g[fin] - r32[fin]) / np.maximum(1, np.abs(r32[fin]))
    f = fin & np.isfinite(r64)
    sc = np.maximum(1, np.abs(r64[f]))
    e_g = np.abs(g[f] - r64[f])
    e_o = np.abs(r32[f] - r64[f])
    ok = e_g <= 1e-5 * sc + 2 * (e_o + sens[f])
    wc = sens[f] / sc <= 2.5e-6
    e_s = np.abs(g[f] - r32[f]) / np.maximum(1, np.abs(r32[f]))
    nll_g = nll_from_sum(float(g.sum()), g.size)
    nll_o = O.nll(r32)
    worst = int(np.argmax(e_g / sc)) if f.any() else -1
    return {
        "rows": int(len(rows)),
        "finiteness_mismatches": mism,
        "strict_max_rel_err_vs_oracle32_all_rows": float(e_all.max()) if e_all.size else None,
        "well_conditioned_rows": int(wc.sum()),
        "strict_max_rel_err_vs_oracle32_well_conditioned": float(e_s[wc].max()) if wc.any() else None,
        "gpu_max_rel_err_vs_fp64": float((e_g / sc).max()) if f.any() else None,
        "oracle32_max_rel_err_vs_fp64": float((e_o / sc).max()) if f.any() else None,
        "gpu_mean_rel_err_vs_fp64": float((e_g / sc).mean()) if f.any() else None,
        "oracle32_mean_rel_err_vs_fp64": float((e_o / sc).mean()) if f.any() else None,
        "within_conditioned_tolerance": float(ok.mean()) if f.any() else None,
        "worst_row_vs_fp64": int(rows[np.flatnonzero(f)[worst]]) if worst >= 0 else None,
        "nll_gpu": nll_g,
        "nll_oracle32": nll_o,
        "nll_rel_diff": abs(nll_g - nll_o) / max(1.0, abs(nll_o)),
    }


def inverse_parity(spec, variables, z, c, xg, rows):
    """GPU inverse rows vs the oracle's Chain.inverse (fp32 and fp64):
    max |err| / max(1, |x|) per element."""
    from oracle import zf_oracle as O

    zs, cs = z[rows], (None if c is None else c[rows])
    g = xg[rows].astype(np.float64)
    r32 = O.flow_inverse(spec, variables, zs, cs).astype(np.float64)
    r64 = O.flow_inverse(spec, variables, zs, cs, dtype=np.float64)
    f = np.isfinite(r32) & np.isfinite(g) & np.isfinite(r64)
    sc = np.maximum(1, np.abs(r64[f]))
    return {
        "rows": int(len(rows)),
        "finiteness_mismatches": int((np.isfinite(r32) != np.isfinite(g)).sum()),
        "max_rel_err_vs_oracle32": float((np.abs(g[f] - r32[f]) / np.maximum(1, np.abs(r32[f]))).max()),
        "gpu_max_rel_err_vs_fp64": float((np.abs(g[f] - r64[f]) / sc).max()),
        "oracle32_max_rel_err_vs_fp64": float((np.abs(r32[f] - r64[f]) / sc).max()),
    }


def config_block(names, steps, warmup):
    """Every other BASELINE config on this GPU (configs[2]-[4]; cfg5 at its
    per-GPU shard of the 8-GPU batch), each timed over `steps` launches with
    HIP events and checked against the oracle on a strided row sample."""
    from zenflow_amd import _lib as L
    from zenflow_amd._lib import DeviceArray, Event
    from zenflow_amd.engine import _latent_code

    lib = L.load_library()
    out = {}
    for name in names:
        t_start = time.perf_counter()
        D, C, K, layers, nL, latent, mode, act = workload(name)
        N = 1 << 20
        flow, variables, x, c = make_workload(name, N)
        prog = flow.bind(variables, D, C).program
        xd = DeviceArray.from_numpy(x)
        cd = DeviceArray.from_numpy(c) if C else None
        res = DeviceArray((N,)) if mode == "log_prob" else DeviceArray((N, D))
        seed = 1234

        def run():
            if mode == "log_prob":
                prog.log_prob(xd, cd, out=res)
            elif mode == "inverse":
                prog.inverse(xd, cd, out=res)
            else:
                prog.sample(N, seed, cd, out=res)

        for _ in range(warmup):
            run()
        L.synchronize()
        evs = [(Event(), Event()) for _ in range(steps)]
        t0 = time.perf_counter()
        for a, b in evs:
            a.record()
            run()
            b.record()
        L.synchronize()
        wall = (time.perf_counter() - t0) / steps
        kavg = float(np.mean([a.elapsed_ms(b) for a, b in evs])) * 1e-3
        fps = flops_per_sample(name)
        peak, _ = SPLIT_PEAKS.get(prog.kernel_variant, (PEAK_FP32_MFMA_TFLOPS, ""))
        entry = {"mode": mode, "rows": N, "kernel": prog.kernel_variant, "ms_per_step": wall * 1e3,
                 "kernel_us": kavg * 1e6, "samples_per_s": N / wall,
                 "achieved_tflops": fps * N / kavg / 1e12, "frac": fps * N / kavg / 1e12 / peak}
        spec = oracle_spec(name)
        rows = sample_rows(N, 4096 if name != "cfg5" else 2048)
        if mode == "log_prob":
            entry["parity"] = logprob_parity(spec, variables, x, c, res.numpy(), rows)
        elif mode == "inverse":
            entry["parity"] = inverse_parity(spec, variables, x, c, res.numpy(), rows)
        else:  # Flow.sample: the same device latent draw through the oracle's inverse
            code, param = _latent_code(prog.latent)
            z = DeviceArray((N, D))
            L.check(lib.zf_latent_sample(code, param, seed, z.ptr, N, D, L.stream()), "zf_latent_sample")
            entry["parity"] = inverse_parity(spec, variables, z.numpy(), c, res.numpy(), rows)
        entry["wall_s"] = time.perf_counter() - t_start
        out[name] = entry
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="cfg2", choices=sorted(WORKLOADS))
    ap.add_argument("--rows-log2", type=int, default=None, help="rows per GPU = 2^k (default 20; cfg1: 12)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=24.0)
    ap.add_argument("--no-spline-kernel", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the other BASELINE configs (rank 0, N=1)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch and rendezvous only: rank 0 prints the run's config, no GPU is touched")
    ap.add_argument("--force-rccl", action="store_true", help="RCCL all-reduce even at world size 1 (plumbing check)")
    ap.add_argument("--serial-allreduce", action="store_true",
                    help="NLL all-reduce on the compute stream after every step (no overlap)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher around us: start one fresh process per GPU (before this
        # process touches the GPU) and exit with the worst rank's status
        from zenflow_amd.launch import spawn

        sys.exit(spawn(args.gpus, [str(Path(__file__).resolve()), *sys.argv[1:]]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launch has WORLD_SIZE={world} ranks")
    rdzv = None
    if world > 1:
        from zenflow_amd.launch import FileRendezvous

        rdzv = FileRendezvous.from_env()

    def barrier(tag):
        if rdzv is not None:
            rdzv.barrier(tag)

    name = args.config
    D, C, K, layers, nL, latent, mode, act = workload(name)
    N = 1 << (args.rows_log2 if args.rows_log2 is not None else (12 if mode == "apply" else 20))
    if args.dry_run:
        barrier("dry_run")
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "config": run_config(name, N, world)}), flush=True)
        if rdzv is not None:
            rdzv.close()
        return

    from zenflow_amd import _lib as L
    from zenflow_amd._lib import DeviceArray, Event
    from zenflow_amd.dist import DataParallelLogProb, DeviceLogProbStep, RcclCommunicator

    L.ensure_device()
    flow, variables, x, c = make_workload(name, N, rank)
    bf = flow.bind(variables, D, C)
    prog = bf.program
    xd = DeviceArray.from_numpy(x)
    cd = DeviceArray.from_numpy(c) if C else None
    out = DeviceArray((N,)) if mode == "log_prob" else DeviceArray((N, D))
    lib = L.load_library()
    comm = None
    if world > 1 or args.force_rccl:
        bcast = (lambda b: b) if rdzv is None else (lambda b: rdzv.broadcast_bytes(b, tag="rccl_uid"))
        comm = RcclCommunicator(rank, world, bcast, force=args.force_rccl)
    dp = DataParallelLogProb(DeviceLogProbStep(prog, N), comm, overlap=not args.serial_allreduce)

    def step(ev=None):
        if mode == "log_prob":
            dp.step(xd, cd, out, ev)
        elif mode == "apply":  # Flow.__call__ through apply: host x in, host log_prob out
            if ev is not None:
                ev[0].record()
            flow.apply(variables, x, c)
            if ev is not None:
                ev[1].record()
        elif mode == "sample":
            if ev is not None:
                ev[0].record()
            prog.sample(N, 1234 + rank, cd, out=out)
            if ev is not None:
                ev[1].record()
        else:
            if ev is not None:
                ev[0].record()
            prog.inverse(xd, cd, out=out)
            if ev is not None:
                ev[1].record()

    def sync_all():  # the library stream and, with overlap, the comm stream
        L.check(lib.zf_device_synchronize(), "device_synchronize")

    for _ in range(args.warmup):
        step()
    sync_all()
    evs = [(Event(), Event()) for _ in range(args.steps)]
    barrier("start")
    sync_all()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    sync_all()
    t1 = time.perf_counter()
    barrier("stop")
    elapsed = t1 - t0
    if rdzv is not None:
        elapsed = rdzv.max(elapsed, "elapsed")
    kern_ms = [a.elapsed_ms(b) for (a, b) in evs]
    kavg = float(np.mean(kern_ms))
    ms_per_step = 1e3 * elapsed / args.steps
    total = N * world * args.steps
    value = total / elapsed

    fps = flops_per_sample(name)
    achieved = fps * N / (kavg * 1e-3) / 1e12
    variant = prog.kernel_variant
    kernel_name = "flow_kernel_x3" if variant in SPLIT_PEAKS else "flow_kernel"
    peak, peak_basis = SPLIT_PEAKS.get(variant, (PEAK_FP32_MFMA_TFLOPS, "fp32 dense MFMA peak"))
    pmc = load_pmc(kernel_name) if rank == 0 else {}
    traffic = pmc.get("hbm_bytes_per_launch")
    held_ghz = None
    if pmc.get("kernel_cycles") and pmc.get("avg_duration_us_trace"):
        held_ghz = pmc["kernel_cycles"] / (pmc["avg_duration_us_trace"] * 1e3)
    result = {
        "metric": "log_prob samples/sec (+ NLL match) 4D 16-knot 4-layer flow, batch 2^20"
        if name == "cfg2" else ("log_prob samples/sec through Flow.apply (host in/out)" if mode == "apply"
                                else f"{mode} samples/sec ({name})"),
        "value": value,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32" if variant not in SPLIT_PEAKS else f"fp32 ({variant} split MFMA, fp32 accumulate)",
        "data": "synthetic: x ~ N(0, I) per rank; random-init weights (flax default initialisers) "
                "+ one train-mode pass for ShiftBounds/BatchNorm statistics",
        "config": dict(run_config(name, N, world), kernel=variant),
        "roofline": {
            "bound": "mfma",
            "achieved": achieved,
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": achieved / peak,
            "traffic": traffic,
            "kernel": f"{kernel_name} (avg {kavg * 1e3:.1f} us over {args.steps} timed launches, HIP events)",
            "kernel_us": kavg * 1e3,
            "alg_flops_per_sample": fps,
            "peak_basis": peak_basis,
            "frac_of_fp32_mfma_peak": achieved / PEAK_FP32_MFMA_TFLOPS,
            "mfma_busy": pmc.get("mfma_busy"),
            # the shader clock the kernel held in the committed counter pass
            # (GRBM_GUI_ACTIVE / 8 XCDs per launch / the trace's average
            # duration) and frac at that clock: frac = mfma-pipe share x the
            # clock ratio (the peak assumes 2.4 GHz)
            "held_clock_ghz": held_ghz,
            "frac_at_held_clock": (achieved / peak) * (PEAK_CLOCK_GHZ / held_ghz) if held_ghz else None,
            "valu_active": pmc.get("valu_active"),
            "valu_mfma_coexec": pmc.get("valu_mfma_coexec"),
            "pmc_source": pmc.get("source"),
            "pipe_source": pmc.get("pipe_source"),
            "pmc_grid": pmc.get("grid"),
        },
    }
    if mode == "log_prob":
        result["nll"] = dp.nll(N * world)
        result["config"]["communicator_ranks"] = comm.world if comm is not None else 1
    if mode == "apply":
        # the same batch resident in HBM (fused kernel + NLL reduce only), and
        # Flow.sample through apply (latent drawn on the device, host out)
        rate = {}
        res_out = DeviceArray((N,))
        for tag in ("log_prob_resident_hbm", "sample_apply"):
            def one():
                if tag == "sample_apply":
                    flow.apply(variables, N, method="sample", seed=7)
                else:
                    dp.step(xd, cd, res_out)
            for _ in range(3):
                one()
            sync_all()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                one()
            sync_all()
            rate[tag] = N * args.steps / (time.perf_counter() - t0)
        result["apply_path"] = {"log_prob_apply_samples_per_s": value, **{k + "_samples_per_s": v for k, v in rate.items()},
                                "note": "value = Flow.apply(variables, x_host) per step: host->device copy, fused "
                                        "kernel, device->host copy and Python dispatch; cached device program"}
    if not args.no_spline_kernel and rank == 0:
        result["spline_kernel"] = spline_kernel_roofline(N, 2, K, args.steps)
        if K != 32:  # K1 at 32 knots too (the two-lanes-per-item kernel)
            result["spline_kernel_k32"] = spline_kernel_roofline(N, 2, 32, args.steps)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        spec = oracle_spec(name)
        if mode in ("log_prob", "apply"):
            cb, outs = cpu_baseline(spec, variables, x, c, args.cpu_budget)
            lp = out.numpy() if mode == "log_prob" else flow.apply(variables, x, c)
            errs, mism, ref_sum, gpu_sum, nrows = [], 0, 0.0, 0.0, 0
            for lo, ref in outs:
                g = lp[lo : lo + ref.shape[0]]
                f = np.isfinite(ref) & np.isfinite(g)
                mism += int((np.isfinite(ref) != np.isfinite(g)).sum())
                errs.append(np.abs(g[f] - ref[f]) / np.maximum(1, np.abs(ref[f])))
                ref_sum += float(ref.astype(np.float64).sum())
                gpu_sum += float(g.astype(np.float64).sum())
                nrows += ref.shape[0]
            e = np.concatenate(errs)
            from zenflow_amd.dist import nll_from_sum

            nll_g, nll_o = nll_from_sum(gpu_sum, nrows), nll_from_sum(ref_sum, nrows)
            result["parity"] = {"rows_checked": int(e.size + mism), "max_rel_err_vs_oracle32": float(e.max()),
                                "p999_rel_err": float(np.quantile(e, 0.999)), "mean_rel_err": float(e.mean()),
                                "finiteness_mismatches": mism, "tolerance": 1e-5,
                                "nll_checked_rows": {"gpu": nll_g, "oracle32": nll_o,
                                                     "rel_diff": abs(nll_g - nll_o) / max(1.0, abs(nll_o))},
                                "fp64_subset": logprob_parity(spec, variables, x, c, lp, sample_rows(N, 8192))}
            result["cpu_baseline"] = cb
            result["speedup_vs_cpu"] = value / cb["value"]
    if rank == 0 and world == 1 and name == "cfg2" and not args.no_configs:
        # every other BASELINE config with its parity, in the same driver-run record
        result["configs"] = config_block(["cfg3", "cfg3s", "cfg4", "cfg5"], min(args.steps, 10), 2)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if comm is not None:
        comm.close()
    if rdzv is not None:
        rdzv.close()


if __name__ == "__main__":
    main()
