#!/usr/bin/env python3
"""Benchmark: sequence-timesteps/s of batched fwd-bwd smoothing (BASELINE.json).

One "step" = one pass of the hot path (nipamd_fb: forward_backward_inference,
src/nip.c:1320, batched) over one batch of B synthetic sequences x T time
slices resident in HBM -- SURVEY 8(d) config 2: HMM-shaped DBN with 16 hidden
and 16 observed states, B = 4096 sequences per GPU, T = 1024.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload W]

N > 1: one process per GPU.  Run directly with --gpus N, bench.py starts
``python -m torch.distributed.run --nproc-per-node N`` on itself as a child
process (before anything touches the GPU) and exits with its code; under a
launcher it checks WORLD_SIZE == N and refuses to run otherwise.  fb-style
workloads shard sequences with no data-path collective (RCCL only for the
barrier and the max-over-ranks timing, "scaling": "weak"); the em workload
 exchanges one packed all-gather per EM iteration.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from nip_amd import synth  # noqa: E402  (numpy only; the HIP library loads on first use)

METRIC = "sequence-timesteps/s fwd-bwd smoothing, 16-state DBN; 1/2/4/8-GPU scaling"
HBM_PEAK_GBS = 8000.0            # MI355X spec (MI355X_MICROARCH.md chip table)


def algorithmic_bytes_per_seq_step(N: int, n_obs: int = 1, posterior: bool = True) -> int:
    """What the path must move per sequence-timestep:
    the int32 observations read once (4 B per observed variable), one N-wide
    fp64 interface message written and read back (alpha for t < T/2, beta for
    t >= T/2: 2 x 8N B), the N-wide fp64 posterior written (8N B, fb only)."""
    return 4 * n_obs + 2 * 8 * N + (8 * N if posterior else 0)


# name -> (spec builder, observed vars, query var, default B, T)
WORKLOADS = {
    "fb": ("config2", lambda a: synth.hmm_spec(a.N, a.M), ["M1"], "P1", 4096, 1024),
    "estep": ("config4", lambda a: synth.hmm_spec(a.N, a.M), ["M1"], "P1", 131072, 1024),
    "config3": ("config3", lambda a: synth.demo1_spec(32), ["A1", "B1"], "C1", 65536, 256),
    "config5": ("config5", lambda a: synth.wide_spec(64, 16), ["O1"], "X1", 256, 128),
    "generate": ("config2", lambda a: synth.hmm_spec(a.N, a.M), ["M1"], "P1", 65536, 1024),
    "em": ("config4", lambda a: synth.hmm_spec(a.N, a.M), ["M1"], "P1", 131072, 1024),
    # the general join-tree engine (not a BASELINE config): a factorial HMM,
    # two 4-state chains with one 16-state observation of both (interface {X1, Y1})
    "jtree": ("general", lambda a: synth.factorial_spec(4, 4, 16), ["O1"], "X1", 4096, 1024),
    # the same slice as a joint-interface chain (16 joint states) on the
    # matrix-core chain kernels -- what the automatic engine choice runs
    "joint": ("general", lambda a: synth.factorial_spec(4, 4, 16), ["O1"], "X1", 4096, 1024),
}


def host_info():
    """CPU model and the cores the baseline may use (the GPU box grants 16
    per GPU: OMP_NUM_THREADS; os.cpu_count() shows the whole machine)."""
    model = platform.processor() or "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
    return model, cores, os.cpu_count()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_or_check(args, argv):
    """--gpus N > 1 without a launcher: run N ranks under torch.distributed.run
    as a child process and exit with its code (nothing here has touched the
    GPU).  Under a launcher: WORLD_SIZE must equal --gpus."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
               "--master-port", str(free_port()), os.path.abspath(__file__), *argv]
        sys.exit(subprocess.call(cmd))
    world = int(world_env or "1")
    if world != args.gpus:
        sys.exit("bench: --gpus %d but WORLD_SIZE=%d; refusing to report a different world size"
                 % (args.gpus, world))
    return world


def cpu_baseline_generate(nodes, pots, T, budget_s: float = 12.0):
    """The reference's generate_data (oracle/_ref harness: nip.c's sampling
    loop over the reference's own join-tree code) on this host, one core,
    series of the bench length until the budget is spent."""
    from oracle import bind
    orc = bind.RefHarness(synth.spec_to_replay(nodes, pots), cards=[n[1] for n in nodes])
    t0 = time.perf_counter()
    n = 0
    while True:
        orc.generate(12345 + n, 1, T)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": n * T / el, "unit": "sequence-timesteps/s", "cores": 1, "kind": "reference",
            "sample": "%d series x T=%d, generate_data (nip.c:2325-2478 loop over the reference's "
                      "nippotential/nipjointree code compiled from /root/reference sources), gcc -O2, "
                      "%.1f s" % (n, T, el)}


def cpu_baseline(nodes, pots, obs, ov, q, budget_s: float = 12.0, t_sample: int = 0):
    """Reference-equivalent CPU path on this host over a bounded sample of the
    bench workload: the C restatement of forward_backward_inference
    (oracle/nip_oracle.c, bit-identical to the reference's own code on every
    golden case) with OpenMP over sequences on all granted cores, one
    sequence per thread.  Where oracle/_ref exists (built in
    the build container), the reference's own compiled code is also timed
    on one core and r = port/ref per-core throughput is reported.  ov / q
    are variable indices in declaration order; t_sample > 0 times only the
    first t_sample slices of each sequence (config 5's 16.7M-entry clique)."""
    from oracle import bind
    import nip_amd
    cpu, cores, ncpu = host_info()
    T = t_sample or obs.shape[1]
    orc = bind.PortOracle(nip_amd.Model.from_spec(nodes, pots).desc())
    # size the sample: one sequence on one thread first
    t0 = time.perf_counter()
    orc.fb(obs[0][:T], ov, [q])
    one = max(time.perf_counter() - t0, 1e-6)
    n = int(max(cores, min(obs.shape[0], budget_s / one * cores)))
    n = max(cores, (n // cores) * cores)
    sample = np.ascontiguousarray(obs[:n, :T])
    t0 = time.perf_counter()
    orc.fb_batch(sample, ov, [q], nthreads=cores)
    el = time.perf_counter() - t0
    rec = {"value": n * T / el, "unit": "sequence-timesteps/s", "cores": cores, "kind": "port",
           "cpu_model": cpu, "host_cpus": ncpu,
           "sample": "%d sequences x T=%d of the bench workload, forward_backward_inference with ll, "
                     "C restatement (oracle/nip_oracle.c, gcc -O2) with OpenMP over %d threads, "
                     "%.1f s" % (n, T, cores, el)}
    try:
        if bind.ref_available():
            ref = bind.RefHarness(synth.spec_to_replay(nodes, pots), cards=[x[1] for x in nodes])
            k, t0 = 0, time.perf_counter()
            while True:
                ref.fb(obs[k][:T], ov, [q])
                k += 1
                if time.perf_counter() - t0 >= budget_s / 4 or k >= obs.shape[0]:
                    break
            ref_rate = k * T / (time.perf_counter() - t0)
            rec["reference_1core"] = ref_rate
            rec["r_port_over_ref_per_core"] = (rec["value"] / cores) / ref_rate
    except Exception as e:  # the reference build is optional on the GPU box
        rec["reference_1core_error"] = str(e)[:200]
    return rec


def load_traffic(workload: str):
    """HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")   # profiles/summarize.py
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get("entries", {}).get(workload)
        if e:
            return e.get("hbm_bytes_per_launch")
    except Exception:
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0, help="sequences per GPU (0: the workload's)")
    ap.add_argument("--T", type=int, default=0, help="time slices (0: the workload's)")
    ap.add_argument("--N", type=int, default=16)
    ap.add_argument("--M", type=int, default=16)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="fb",
                    help="fb: the headline metric (config 2 smoothing); estep: one batched "
                         "e_step (config 4 per-GPU shard: counts + ll, no posterior write); "
                         "em: config 4, one step = one em_learn iteration (m_step, e_step of "
                         "the shard, the packed all-gather over RCCL, finalize); "
                         "config3: demo1 @ 32 states smoothing; config5: wide-clique smoothing; "
                         "jtree: a factorial HMM on the general join-tree engine; "
                         "joint: the same slice as a joint-interface chain")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the output sanity check (ablation builds)")
    args = ap.parse_args()
    world = launch_or_check(args, sys.argv[1:])

    import torch
    import torch.distributed as dist
    import nip_amd

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    cfg, spec, ov_names, q_name, B0, T0 = WORKLOADS[args.workload]
    B, T = args.batch or B0, args.T or T0
    nodes, pots = spec(args)
    model = nip_amd.Model.from_spec(nodes, pots)
    ov, q = [model.variable(v) for v in ov_names], model.variable(q_name)
    if args.workload == "jtree":
        model.set_engine(nip_amd.ENGINE_JTREE)     # the joint-interface chain would take it otherwise
    N, M = model.card(q), model.card(ov[0])
    obs_np = np.concatenate([synth.observations(B, T, model.card(v), seed=1 + 7919 * rank + 104729 * i)
                             for i, v in enumerate(ov)], axis=2)
    obs = torch.from_numpy(obs_np).to(dev)
    ll = torch.empty((B,), dtype=torch.float64, device=dev)
    st = torch.empty((B,), dtype=torch.int32, device=dev)
    if args.workload == "generate":
        sample = torch.empty((B, T, model.num_vars), dtype=torch.int32, device=dev)
        st.zero_()
        ll.zero_()

        def step():
            nip_amd.generate_data(model, 12345 + rank, B, T, sample)
    elif args.workload == "em":
        from nip_amd import em as nem
        group = dist.group.WORLD if world > 1 else None
        em_state = {"params": synth.uniform01(2024, model.param_size()) + 0.05, "ll": [],
                    "exchange_ms": []}

        def step():
            tm = {}
            p, l, bad = nem.iteration(model, em_state["params"], obs, ov, group, timing=tm)
            if bad:
                raise SystemExit("bench: e_step BAD_LUCK on synthetic data")
            em_state["params"] = p
            em_state["ll"].append(l)
            em_state["exchange_ms"].append(tm.get("exchange_ms", 0.0))
    elif args.workload != "estep":
        post = torch.empty((B, T, N), dtype=torch.float64, device=dev)

        def step():
            nip_amd.forward_backward_inference(model, obs, ov, [q], post, ll, st)
    else:
        counts = torch.ones((model.param_size(),), dtype=torch.float64, device=dev)

        def step():
            nip_amd.e_step(model, obs, ov, counts, ll, st)

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[dev.index])
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record()
        step()
        evs[i][1].record()
    barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    if args.workload == "em":
        ll.zero_()
        st.zero_()
    if not args.no_check and (not bool(torch.isfinite(ll).all()) or int(st.abs().sum()) != 0):
        raise SystemExit("bench: non-finite log-likelihood / zero-mass status on synthetic data")

    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    units = B * T * args.steps * world
    value = units / elapsed
    bpu = algorithmic_bytes_per_seq_step(N, len(ov), args.workload not in ("estep", "em"))
    narrow = N <= 16 and len(ov) <= 1
    if not narrow and N <= 32 and os.environ.get("NIPAMD_FB_KERNEL") != "wide":
        kname = "chain_mfma_wide_kernel<%d>" % (1 if N <= 16 else 2)
    elif not narrow:
        kname = ("chain_wide4_kernel" if N > 32 and os.environ.get("NIPAMD_WIDE_KERNEL") != "wave1"
                 else "chain_wide_kernel<%d>" % (16 if N <= 16 else 32 if N <= 32 else 64))
    elif os.environ.get("NIPAMD_FB_KERNEL") == "scratch":
        kname = "chain_fb_mfma_kernel"
    elif os.environ.get("NIPAMD_FB_KERNEL") != "dpp":
        kname = "chain_fb_ckpt_kernel"     # 16-state posteriors (config 2); else chain_fb_mfma_kernel
    else:
        kname = "chain_kernel<false>"
    metric = METRIC
    if args.workload == "fb":
        workload = "config2: HMM-shaped DBN, %d hidden x %d observed states, B=%d seq/GPU x T=%d" % (
            N, M, B, T)
    elif args.workload == "estep":
        kname = ("chain_fb_mfma_kernel<true, true>" if os.environ.get("NIPAMD_ESTEP_KERNEL") == "mfma"
                 else "chain_kernel<true>") + " + tree64 + finalize"
        workload = "config4 shard: e_step of HMM-shaped DBN, %d hidden x %d observed, B=%d seq/GPU x T=%d" % (
            N, M, B, T)
        metric = "sequence-timesteps/s batched e_step (EM expected counts), 16-state DBN"
    elif args.workload == "em":
        kname = "chain_kernel<true> + tree64 + finalize"
        workload = ("config4: em_learn iterations of HMM-shaped DBN, %d hidden x %d observed, "
                    "B=%d seq/GPU x T=%d, %d GPU(s), one packed RCCL all-gather per iteration" % (
                        N, M, B, T, world))
        metric = "sequence-timesteps/s em_learn (E-step + exchange + M-step per iteration), 16-state DBN"
    elif args.workload == "generate":
        kname = "generate_kernel"
        bpu = 4 * model.num_vars       # the int32 draws written; the tables stay in cache
        workload = "generate_data: HMM-shaped DBN, %d hidden x %d observed states, B=%d series/GPU x T=%d" % (
            N, M, B, T)
        metric = "sequence-timesteps/s generate_data (sampling), 16-state DBN"
    elif args.workload == "jtree":
        kname = "jt_filter_kernel + jt_post_kernel"
        bpu = 4 + 8 * N                # I/O only: the obs read, the posterior written
        workload = ("general join-tree engine: factorial HMM, X and Y 4 states each, O1 16 states of both, "
                    "X1 posterior, B=%d seq/GPU x T=%d" % (B, T))
        metric = "sequence-timesteps/s fwd-bwd smoothing, factorial HMM (general join-tree engine)"
    elif args.workload == "joint":
        K = 16                         # joint interface states (X1, Y1)
        kname = "chain_fb_ckpt_kernel + derive_kernel"
        # the chain kernel's bytes at K states, then the derive pass: the joint
        # posterior read back, X1's marginal written
        bpu = algorithmic_bytes_per_seq_step(K, len(ov), True) + 8 * K + 8 * N
        workload = ("joint-interface chain: factorial HMM, X and Y 4 states each, O1 16 states of both, "
                    "X1 posterior, B=%d seq/GPU x T=%d" % (B, T))
        metric = "sequence-timesteps/s fwd-bwd smoothing, factorial HMM (joint-interface chain kernels)"
    elif args.workload == "config3":
        workload = "config3: demo1.net structure, 5 vars x 32 states, A1 B1 observed, C1 posterior, " \
                   "B=%d seq/GPU x T=%d" % (B, T)
        metric = "sequence-timesteps/s fwd-bwd smoothing, demo1 @ 32 states"
    else:
        workload = "config5: wide clique {X0,Y1,Z1,X1} 64^4 entries, O1 16 states observed, X1 posterior, " \
                   "B=%d seq/GPU x T=%d" % (B, T)
        metric = "sequence-timesteps/s fwd-bwd smoothing, wide-clique DBN (64^4 in-clique)"
    achieved = bpu * B * T / (kern_ms * 1e-3) / 1e9
    traffic = load_traffic(workload)
    if rank == 0:
        rec = {
            "metric": metric, "value": value, "unit": "sequence-timesteps/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": workload, "B_per_gpu": B, "T": T, "hidden_states": N,
                       "observed_states": M, "observed_vars": len(ov), "parallelism": "dp%d" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "kernel": kname,
                         "kernel_ms": kern_ms, "bytes_per_unit": bpu},
        }
        if args.workload == "em":
            rec["em"] = {"iterations_timed": args.steps, "ll_per_iteration": em_state["ll"][-args.steps:],
                         "exchange_ms_median": float(np.median(em_state["exchange_ms"][-args.steps:])),
                         "exchange_bytes_per_rank": 8 * (model.param_size() + 2),
                         "note": "kernel_ms is the whole iteration on the launch stream "
                                 "(e_step kernels, exchange, finalize, host m_step)"}
        if args.workload == "jtree":
            rec["roofline"]["note"] = "bytes are the request's I/O only; the engine is latency-bound (DESIGN.md 4)"
        if world == 1 and args.workload in ("fb", "config3", "config5"):
            # PCIe-inclusive figure: the same batch from host
            # buffers through nipamd_fb_host (H2D obs, kernels, D2H posteriors)
            host_obs = np.ascontiguousarray(obs_np)
            nip_amd.forward_backward_inference_host(model, host_obs, ov, [q])
            t1 = time.perf_counter()
            nip_amd.forward_backward_inference_host(model, host_obs, ov, [q])
            el1 = time.perf_counter() - t1
            rec["pcie_inclusive"] = {"value": B * T / el1, "unit": "sequence-timesteps/s", "ms": el1 * 1e3,
                                     "note": "host buffers in and out (pageable), one call; not the headline"}
        if args.workload == "config5":
            # the in-clique marginalisation: 64^4 entries summed over the hidden
            # parents on the GPU (fold.hip), once per model version
            fms, fby = [], 0.0
            for _ in range(5):
                _, ms_f, fby = model.fold()
                fms.append(ms_f)
            fk = float(np.median(fms))
            rec["fold"] = {"kernel": "fold_kernel", "kernel_ms": fk, "bytes": fby,
                           "roofline": {"bound": "hbm", "achieved": fby / (fk * 1e-3) / 1e9,
                                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                        "frac": fby / (fk * 1e-3) / 1e9 / HBM_PEAK_GBS},
                           "note": "A[x][y] = sum over Y1, Z1 of the 134 MB clique x priors, per model version"}
        if world == 1 and not args.no_cpu_baseline and args.workload == "generate":
            rec["cpu_baseline"] = cpu_baseline_generate(nodes, pots, T)
        elif world == 1 and not args.no_cpu_baseline and args.workload not in ("estep", "em"):
            names = [n[0] for n in nodes]
            rec["cpu_baseline"] = cpu_baseline(
                nodes, pots, obs_np, [names.index(v) for v in ov_names], names.index(q_name),
                t_sample=2 if args.workload == "config5" else 0)
        print(json.dumps(rec))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
