#!/usr/bin/env python3
"""Benchmark: sequence-timesteps/s of batched fwd-bwd smoothing (BASELINE.json).

One "step" = one pass of the hot path (nipamd_fb: forward_backward_inference,
src/nip.c:1320, batched) over one batch of B synthetic sequences x T time
slices resident in HBM -- SURVEY 8(d) config 2: HMM-shaped DBN with 16 hidden
and 16 observed states, B = 4096 sequences per GPU, T = 1024.  The same JSON
line carries a `secondary` object with SURVEY 8(d)'s other GPU configs timed
the same way in the same run: config 3 (demo1 @ 32 states, 65536 x 256),
config 4 (one em_learn iteration over the 131072 x 1024 per-GPU shard) and
config 5 (the 64^4 wide clique, 256 x 128).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload W] [--no-secondary]

N > 1: one process per GPU.  Run directly with --gpus N, bench.py starts
``python -m torch.distributed.run --nproc-per-node N`` on itself as a child
process (before anything touches the GPU) and exits with its code; under a
launcher it checks WORLD_SIZE == N and refuses to run otherwise.  fb-style
workloads shard sequences with no data-path collective (RCCL only for the
barrier and the max-over-ranks timing, "scaling": "weak"); the em workload
 exchanges one packed all-gather per EM iteration.
Rank 0 prints one JSON line.

Roofline accounting:
  roofline.achieved   the bytes the dominant kernel's algorithm moves per
                      sequence-timestep (`bytes_per_unit`, e.g. 196 B for the
                      checkpoint kernel: obs + checkpoints written and read +
                      posterior) x units / kernel time (HIP events on the launch
                      stream) -- never bytes the kernel does not move
  roofline.primary    SURVEY 8(d)'s per-unit figure (392 B at config 2, with
                      the alpha/beta round trip) at the same time: a like-for-
                      like comparison across kernels, NOT delivered bandwidth
  roofline.latency    the second roof: the filters' dependency chain, T steps
                      of the measured minimal step (profiles/r03/r03_mb_lat.txt)
                      per block round, against the kernel time
  roofline.traffic    HBM bytes per step from the committed rocprofv3 PMC pass
                      (profiles/pmc_traffic.json, gfx950 FETCH_SIZE x2)
"""
from __future__ import annotations

import argparse
import json
import os
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
N_CU = 256
# Dependency-chain floors of the matrix-core filters, measured by
# profiles/r03/mb_lat.hip (one wave per CU, s_memtime cycles; r03x_mb_lat.txt):
# kernel -> (cycles per filter step, sequences per block, blocks resident per CU)
LATENCY_STEP = {
    # 4 chained v_mfma_f64_16x16x4 and the step's evidence multiply on the
    # VALU between them (V4: the recursion's own dependency chain, 424 cycles
    # in round 6's profiles/r06/gpu/r06a_mb_lat6.txt, 464 in round 3's build;
    # the MFMAs alone, V2, take 328)
    "chain_fb_ckpt_kernel": (424.0, 16, 1),
    "chain_fb_ckpt_kernel<proj>": (424.0, 16, 1),
    "chain_fb_mfma_kernel": (424.0, 16, 1),
    "chain_mfma_wide_kernel<1>": (424.0, 32, 1),       # two groups of 16 per block, concurrently
    "chain_mfma_wide_kernel<2>": (1136.1, 32, 1),      # 2 x 8 chained MFMAs, interleaved (V3); two groups of 16
}
CLOCK_GHZ = 2.39                 # in-kernel clock under the chain loop (s_memtime / s_memrealtime, r03_mb_lat.txt)
MAX_CLOCK_GHZ = 2.4              # MI355X max engine clock (MI355X_MICROARCH.md chip table)

# SURVEY 8(d)'s primary per-unit figures (HBM bytes per sequence-timestep)
PRIMARY_BYTES = {"config2": 392, "config3": 784, "config4": 264, "config5": 1544}


def kernel_bytes(kname: str, N: int, n_obs: int, posterior: bool):
    """Bytes per sequence-timestep the dominant kernel's algorithm moves in HBM,
    and the breakdown."""
    if kname == "chain_fb_ckpt_kernel":
        ck = 8 * N // 4
        return (4 * n_obs + 2 * ck + 8 * N,
                "obs %d + every 4th interface message as a checkpoint (%d written + %d read) + posterior %d"
                % (4 * n_obs, ck, ck, 8 * N))
    if kname.startswith("chain_estep_ck_kernel"):
        # round 6: every 4th forward message (16 states) and its exponent to HBM, read back once
        ck = (8 * 16 + 4) // 4
        return (2 * 4 * n_obs + 2 * ck,
                "obs %d (read by the forward and the backward pass) + every 4th forward message and its "
                "exponent as a checkpoint (%d written + %d read); the recomputed messages and the counts "
                "stay on chip" % (2 * 4 * n_obs, ck, ck))
    post = 8 * N if posterior else 0
    if kname.startswith("chain_fb_ckw_kernel"):
        # round 6: every 4th forward message (32 states) and its exponent to HBM, read back once
        ck = (8 * 32 + 4) // 4
        return (2 * 4 * n_obs + 2 * ck + post,
                "obs %d (read by the forward and the backward pass) + every 4th forward message and its "
                "exponent as a checkpoint (%d written + %d read) + posterior %d"
                % (2 * 4 * n_obs, ck, ck, post))
    if kname.startswith("chain_mfma_wide_kernel") and posterior:
        # both filters read the observation codes from HBM (no LDS staging)
        return (8 * n_obs + 16 * N + post,
                "obs %d (read by both filters) + interface message written and read back (%d + %d) + posterior %d"
                % (8 * n_obs, 8 * N, 8 * N, post))
    return (4 * n_obs + 16 * N + post,
            "obs %d + interface message written and read back (%d + %d)%s"
            % (4 * n_obs, 8 * N, 8 * N, " + posterior %d" % post if post else " (counts stay on chip)"))


# name -> (spec builder, observed vars, query var, default B, T, default steps)
WORKLOADS = {
    "fb": ("config2", lambda a: synth.hmm_spec(a.N, a.M), ["M1"], "P1", 4096, 1024, 20),
    "estep": ("config4", lambda a: synth.hmm_spec(a.N, a.M), ["M1"], "P1", 131072, 1024, 5),
    "config3": ("config3", lambda a: synth.demo1_spec(32), ["A1", "B1"], "C1", 65536, 256, 10),
    "config5": ("config5", lambda a: synth.wide_spec(64, 16), ["O1"], "X1", 256, 128, 20),
    "generate": ("config2", lambda a: synth.hmm_spec(a.N, a.M), ["M1"], "P1", 65536, 1024, 20),
    "em": ("config4", lambda a: synth.hmm_spec(a.N, a.M), ["M1"], "P1", 131072, 1024, 5),
    # the general join-tree engine (not a BASELINE config): a factorial HMM,
    # two 4-state chains with one 16-state observation of both (interface {X1, Y1})
    "jtree": ("general", lambda a: synth.factorial_spec(4, 4, 16), ["O1"], "X1", 4096, 1024, 5),
    # the same slice as a joint-interface chain (16 joint states) on the
    # matrix-core chain kernels -- what the automatic engine choice runs
    "joint": ("general", lambda a: synth.factorial_spec(4, 4, 16), ["O1"], "X1", 4096, 1024, 20),
    # demo1's structure (6 states) with its hidden parent D1 observed: no
    # interface-chain plan; the evidence-indexed chain (opchain.hip) by default,
    # the general join-tree engine as "opchain_jt"
    "opchain": ("general", lambda a: synth.demo1_spec(6), ["A1", "B1", "D1"], "C1", 4096, 1024, 20),
    "opchain_jt": ("general", lambda a: synth.demo1_spec(6), ["A1", "B1", "D1"], "C1", 4096, 1024, 2),
    # the same request at 20 states (a 20-state joint interface, 9261
    # evidence combinations): the wide operator chain (op_wide_*), and the
    # general engine on a smaller batch ("opchain_wide_jt")
    "opchain_wide": ("general", lambda a: synth.demo1_spec(20), ["A1", "B1", "D1"], "C1", 4096, 1024, 5),
    "opchain_wide_jt": ("general", lambda a: synth.demo1_spec(20), ["A1", "B1", "D1"], "C1", 256, 1024, 1),
    # e_step of config 3's model (demo1 @ 32 states, A1 and B1 observed): the
    # wide chain e_step (estep_wide.hip)
    "estep_config3": ("config3", lambda a: synth.demo1_spec(32), ["A1", "B1"], "C1", 65536, 256, 5),
    # e_step of demo1's structure (16 states: hidden parent D1, children A1, B1)
    # on the chain e_step kernel, and on the general engine ("estep_demo1_jt")
    "estep_demo1": ("general", lambda a: synth.demo1_spec(16), ["A1", "B1"], "C1", 16384, 1024, 5),
    "estep_demo1_jt": ("general", lambda a: synth.demo1_spec(16), ["A1", "B1"], "C1", 4096, 1024, 2),
    # e_step of the opchain workload's request (demo1 @ 6 states, hidden parent
    # D1 observed): the operator chain's e_step, and the general engine's
    "estep_opchain": ("general", lambda a: synth.demo1_spec(6), ["A1", "B1", "D1"], "C1", 4096, 1024, 5),
    "estep_opchain_jt": ("general", lambda a: synth.demo1_spec(6), ["A1", "B1", "D1"], "C1", 4096, 1024, 2),
    # e_step of the opchain_wide request (demo1 @ 20 states, A1 B1 and the
    # hidden parent D1 observed, 9261 evidence combinations): the wide operator
    # chain's e_step (op_wide_msgs_kernel + op_wide_xi_kernel), and the general
    # engine's on a smaller batch
    "estep_opchain_wide": ("general", lambda a: synth.demo1_spec(20), ["A1", "B1", "D1"], "C1", 4096, 1024, 3),
    "estep_opchain_wide_jt": ("general", lambda a: synth.demo1_spec(20), ["A1", "B1", "D1"], "C1", 256, 1024, 1),
}
ESTEP_WORKLOADS = ("estep", "estep_demo1", "estep_demo1_jt", "estep_config3", "estep_opchain", "estep_opchain_jt",
                   "estep_opchain_wide", "estep_opchain_wide_jt")
# the default line: the headline, then these under "secondary" 
SECONDARY = ["config3", "em", "config5", "estep_config3"]


def host_info():
    """CPU model and the cores the baseline may use (the GPU box grants 16
    per GPU: OMP_NUM_THREADS; os.cpu_count() shows the whole machine)."""
    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
    return cores


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


def cpu_baselines(workloads, budget):
    """The reference's own code (and the C port) on the host's granted cores,
    one process per core (oracle/cpu_bench.py), run as a child process
    before this process touches the GPU.  -> {workload: record}."""
    cmap = {"fb": "fb", "config3": "config3", "em": "em", "estep": "em", "config5": "config5",
            "estep_config3": "estep_config3"}
    wl = [cmap[w] for w in workloads if w in cmap]
    if not wl:
        return {}
    cmd = [sys.executable, os.path.join(ROOT, "oracle", "cpu_bench.py"), "--procs", str(host_info()),
           "--budget", str(budget), *wl]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    except Exception as e:
        return {w: {"error": str(e)[:200]} for w in workloads}
    got = {}
    for line in r.stdout.splitlines():
        if line.startswith("{"):
            d = json.loads(line)
            got[d["workload"]] = d
    out = {}
    for w in workloads:
        d = got.get(cmap.get(w))
        if d is None:
            out[w] = {"error": "no baseline: " + r.stderr[-300:]}
            continue
        ref, port = d.get("reference"), d.get("port")
        rec = dict(ref if ref else (port or {}))
        if not rec:
            out[w] = {"error": d.get("error", "no baseline")}
            continue
        rec["cpu_model"], rec["host_cpus"] = d["cpu_model"], d["host_cpus"]
        if ref and port:
            rec["port"] = {k: port[k] for k in ("value", "cores", "kind", "sample")}
            rec["r_port_over_ref"] = port["value"] / ref["value"]
        if not ref:
            rec["note"] = "the reference build (oracle/_ref) is absent: the C port is the baseline"
        out[w] = rec
    return out


def load_entry(workload: str):
    """The committed rocprofv3 PMC pass of a workload (profiles/pmc_traffic.json,
    written by profiles/summarize.py), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            return json.load(f).get("entries", {}).get(workload)
    except Exception:
        return None


def load_traffic(workload: str, single_kernel: bool):
    """HBM bytes per step from the committed rocprofv3 PMC pass (profiles/):
    the dominant kernel's bytes per launch x launches per step when the step
    is that one kernel (fb, config 3, config 5 -- a per-step sum over the
    profiled process would also count the headline's PCIe-inclusive call and
    the output checks), every nipamd kernel's per step otherwise (e_step:
    filters, statistics, trees, finalize)."""
    e = load_entry(workload)
    if e:
        if single_kernel:
            return e.get("hbm_bytes_per_step", e.get("hbm_bytes_per_launch"))
        return e.get("all_kernels_hbm_bytes_per_step", e.get("hbm_bytes_per_step", e.get("hbm_bytes_per_launch")))
    return None


N_SIMD = 4 * N_CU
VALU_ISSUE_CYC = 4.0      # one wave64 VALU instruction per 4 cycles on a 16-lane SIMD (MI355X_MICROARCH.md)
LONE_WAVE_VALU_CYC = 6.27  # f64 VALU issue of a single wave per SIMD, measured (profiles/r04/mb_r64.hip V2)
MFMA_F64_CYC = 64.0       # v_mfma_f64_16x16x4 occupies its SIMD's matrix pipe 64 cycles (profiles/r03/r03_mb_pipe.txt)


def pipe_roof(workload: str, kern_ms: float):
    """The issue roof of the dominant kernel from its committed PMC pass: its
    vector instructions at one per 4 cycles and its matrix-core busy cycles,
    spread over the chip's 1024 SIMDs at the kernel's effective clock, against
    the measured time per step.  frac near 1: the kernel issues as fast as the
    SIMDs can; the gap to 1 is dependency stalls and imbalance."""
    e = load_entry(workload)
    if not e:
        return None
    c = e.get("counters_per_launch", {})
    valu = c.get("SQ_INSTS_VALU")
    if valu is None:
        return None
    mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
    # the part's max engine clock (MI355X_MICROARCH.md: 2400 MHz), not the
    # clock of the counter pass (profiled passes run slower): the
    # smallest floor the instruction counts allow, so frac is a lower bound
    clock = MAX_CLOCK_GHZ
    per = e.get("launches_per_step", 1)
    cyc = (valu * VALU_ISSUE_CYC + (mfma or 0.0)) / N_SIMD
    floor_ms = per * cyc / (clock * 1e9) * 1e3
    return {"bound": "SIMD issue (VALU + matrix core)", "valu_insts_per_launch": valu,
            "mfma_busy_cycles_per_launch": mfma, "launches_per_step": per,
            "clock_ghz": clock, "floor_ms": floor_ms, "frac": floor_ms / kern_ms,
            "source": "profiles/pmc_traffic.json tag %s (rocprofv3 --pmc SQ_INSTS_VALU, SQ_VALU_MFMA_BUSY_CYCLES) "
                      "at the max engine clock" % e.get("tag")}


def row64_issue_roof(B: int, T: int, kern_ms: float):
    """Config 5's filter wave is one sequence's dependency chain on one SIMD:
    its per-step instruction stream (static count of the gfx950 ISA,
    profiles/r04/isa_row64_step.json) at the single-wave issue rates (VALU 4
    cycles, SALU 1, LDS 4) for T steps, one block per CU."""
    p = os.path.join(ROOT, "profiles", "r04", "isa_row64_step.json")
    try:
        with open(p) as f:
            d = json.load(f)
    except Exception:
        return None
    rounds = -(-B // N_CU)

    def floor(valu_cyc):
        cyc = d["valu_per_step"] * valu_cyc + d["salu_per_step"] + d["ds_per_step"] * 4.0
        return cyc, rounds * T * cyc / (CLOCK_GHZ * 1e9) * 1e3

    # a lone wave on its SIMD issues f64 VALU at 6.27 cycles per instruction,
    # not 4 (profiles/r04/mb_r64.hip V2: 64 independent v_fmac_f64_dpp in 401
    # cycles, profiles/r04/gpu/r04h_mb_r64.txt) -- the filter is one sequence's
    # chain, so that is its issue bound; the 4-cycle figure needs two waves
    cyc, floor_ms = floor(LONE_WAVE_VALU_CYC)
    cyc4, floor4 = floor(VALU_ISSUE_CYC)
    return {"bound": "one filter wave's instruction issue (a lone wave's measured f64 VALU rate)",
            "cycles_per_step": cyc, "valu_cycles": LONE_WAVE_VALU_CYC,
            "valu_per_step": d["valu_per_step"], "salu_per_step": d["salu_per_step"],
            "ds_per_step": d["ds_per_step"], "steps": T, "block_rounds": rounds, "clock_ghz": CLOCK_GHZ,
            "floor_ms": floor_ms, "frac": floor_ms / kern_ms,
            "at_4_cycles": {"cycles_per_step": cyc4, "floor_ms": floor4, "frac": floor4 / kern_ms},
            # the same filter code measured alone (timing-only build without the
            # barriers and the partners, NIPAMD_R64_SOLO=1) and in the kernel
            "measured_step_cycles": {"alone_fwd": 566, "alone_bwd": 595, "in_kernel": 667,
                                     "source": "profiles/r06/gpu/r06as, r06av (block stamps)"},
            "source": "profiles/r04/isa_row64_step.json, profiles/r04/gpu/r04h_mb_r64.txt"}


def run_workload(name, args, world, rank, dev, steps, warmup, min_warm_s=0.0):
    """Time `steps` steps of one workload (barrier + synchronize on both sides,
    max over ranks) and build its record."""
    import torch
    import torch.distributed as dist
    import nip_amd

    cfg, spec, ov_names, q_name, B0, T0, _ = WORKLOADS[name]
    headline = name == args.workload
    B = (args.batch if headline and args.batch else B0)
    T = (args.T if headline and args.T else T0)
    nodes, pots = spec(args)
    model = nip_amd.Model.from_spec(nodes, pots)
    ov, q = [model.variable(v) for v in ov_names], model.variable(q_name)
    if name in ("jtree", "opchain_jt", "estep_demo1_jt", "estep_opchain_jt", "opchain_wide_jt", "estep_opchain_wide_jt"):
        model.set_engine(nip_amd.ENGINE_JTREE)     # the chain kernels would take it otherwise
    N, M = model.card(q), model.card(ov[0])
    obs_np = np.concatenate([synth.observations(B, T, model.card(v), seed=1 + 7919 * rank + 104729 * i)
                             for i, v in enumerate(ov)], axis=2)
    obs = torch.from_numpy(obs_np).to(dev)
    ll = torch.empty((B,), dtype=torch.float64, device=dev)
    st = torch.empty((B,), dtype=torch.int32, device=dev)
    em_state = None
    if name == "generate":
        sample = torch.empty((B, T, model.num_vars), dtype=torch.int32, device=dev)
        st.zero_()
        ll.zero_()

        def step():
            nip_amd.generate_data(model, 12345 + rank, B, T, sample)
    elif name == "em":
        from nip_amd import em as nem
        group = dist.group.WORLD if world > 1 else None
        em_state = {"params": synth.uniform01(2024, model.param_size()) + 0.05, "ll": [], "exchange_ms": []}

        def step():
            tm = {}
            p, l, bad = nem.iteration(model, em_state["params"], obs, ov, group, timing=tm)
            if bad:
                raise SystemExit("bench: e_step BAD_LUCK on synthetic data")
            em_state["params"] = p
            em_state["ll"].append(l)
            em_state["exchange_ms"].append(tm.get("exchange_ms", 0.0))
    elif name not in ESTEP_WORKLOADS:
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

    # W warmup steps; the secondary lines (whose W is the bench's own choice)
    # then add steps, at most 64, until about min_warm_s of warmup work has
    # run: the f64-heavy kernels run their first launches at a lower clock
    # while the part settles (config 3: 3.2-3.7 ms before 2.8-2.9 ms,
    # profiles/r04g_timed_region.txt).  The extra count is agreed on before
    # any extra step runs (a MAX over ranks), so steps that contain a
    # collective (em's exchange) stay matched across ranks
    tw = time.perf_counter()
    for _ in range(warmup):
        step()
    nw = warmup
    if min_warm_s > 0.0:
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        nw += 1
        one = max(time.perf_counter() - t1, 1e-6)
        left = min_warm_s - (time.perf_counter() - tw)
        extra = min(63, max(0, int(np.ceil(left / one))))
        if world > 1:
            n_t = torch.tensor([extra], device=dev)
            dist.all_reduce(n_t, op=dist.ReduceOp.MAX)
            extra = int(n_t.item())
        for _ in range(extra):
            step()
        nw += extra
    barrier()
    kname = nip_amd.last_kernel()       # the kernel the engine chose for this request
    # one event pair around the K steps on the launch stream (torch's current
    # stream, which the engine launches on): per-step event packets would sit
    # between the kernels and lengthen the very gaps they measure
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for i in range(steps):
        step()
    ev1.record()
    barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / steps
    if not args.no_check:
        if name == "em":
            # em.iteration raised on any BAD_LUCK series already; its ll (the
            # exchange's tree sum over the shard) must be finite every iteration
            if not np.all(np.isfinite(em_state["ll"])):
                raise SystemExit("bench: non-finite em_learn log-likelihood on synthetic data")
        elif name != "generate" and (not bool(torch.isfinite(ll).all()) or int(st.abs().sum()) != 0):
            raise SystemExit("bench: non-finite log-likelihood / zero-mass status on synthetic data (%s)" % name)
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    units = B * T * steps * world
    value = units / elapsed
    posterior = name not in ESTEP_WORKLOADS + ("em",)
    bpu, bnote = kernel_bytes(kname, N, len(ov), posterior)
    metric = METRIC
    extra = {}
    if name == "fb":
        workload = "config2: HMM-shaped DBN, %d hidden x %d observed states, B=%d seq/GPU x T=%d" % (N, M, B, T)
    elif name == "estep":
        workload = "config4 shard: e_step of HMM-shaped DBN, %d hidden x %d observed, B=%d seq/GPU x T=%d" % (
            N, M, B, T)
        metric = "sequence-timesteps/s batched e_step (EM expected counts), 16-state DBN"
        kname += " + tree64 + finalize"
    elif name == "estep_config3":
        if kname.startswith("chain_estep_ckw_kernel"):
            # round 6: every 4th forward message (32 states) and its exponent to HBM, read back once
            ck = (8 * 32 + 4) // 4
            bpu = 2 * 4 * len(ov) + 2 * ck
            bnote = ("obs %d (read by the forward and the backward pass) + every 4th forward message and its "
                     "exponent as a checkpoint (%d written + %d read); the recomputed messages and the three "
                     "sums stay on chip" % (2 * 4 * len(ov), ck, ck))
            kname += " + tree64 + map finalize"
        elif kname.startswith("chain_estep_mw_kernel"):
            NP = 32
            bpu = 2 * 4 * len(ov) + 2 * 8 * NP + 8
            bnote = ("obs %d (read by both filters) + half of each direction's messages written to the scratch and "
                     "read back (%d + %d) + their exponents 8; the three sums stay on chip"
                     % (2 * 4 * len(ov), 8 * NP, 8 * NP))
            kname += " + tree64 + map finalize"
        elif kname.startswith("chain_msgs_kernel"):
            NP = 16 if N <= 16 else 32 if N <= 32 else 64
            bpu = 3 * 4 * len(ov) + 4 * 8 * NP + 8
            bnote = ("obs %d (read by both filters and the statistics kernel) + alpha^ and beta^ written and read "
                     "(4 x %d) + alpha's exponent written and read 8; the counts stay on chip"
                     % (3 * 4 * len(ov), 8 * NP))
            kname += " + tree64 + map finalize"
        else:
            bpu, bnote = 4 * len(ov), "the request's input only: the engine is latency-bound (DESIGN.md 4)"
        workload = ("config3 e_step: demo1.net structure, 5 vars x 32 states, A1 B1 observed, hidden parent D1, "
                    "B=%d seq/GPU x T=%d (%s)" % (B, T, kname))
        metric = "sequence-timesteps/s batched e_step (EM expected counts), demo1 @ 32 states"
    elif name in ("estep_demo1", "estep_demo1_jt"):
        if kname == "chain_estep16_kernel":
            bpu, bnote = 4 * len(ov) + 2 * 128 + 4, ("obs %d + interface message written and read back (128 + 128) "
                                                     "+ its exponent 4 (counts stay on chip)" % (4 * len(ov)))
            kname += " + tree64 + map finalize"
        else:
            bpu, bnote = 4 * len(ov), "the request's input only: the engine is latency-bound (DESIGN.md 4)"
        workload = ("e_step of demo1's structure, 5 vars x 16 states, hidden parent D1, A1 B1 observed, "
                    "B=%d seq/GPU x T=%d (%s)" % (B, T, kname))
        metric = "sequence-timesteps/s batched e_step, demo1 structure @ 16 states"
    elif name in ("estep_opchain", "estep_opchain_jt"):
        if kname.startswith("op_fb_kernel"):
            K = N                       # the joint interface is C1 alone
            bpu = 4 * len(ov) + 2 * 128 + 8 * K * K + 4 * len(ov)
            bnote = ("obs %d + the 16-wide interface message written and read back (128 + 128) + the step's "
                     "xi weights written and read (%d) + obs re-read by op_xi_kernel %d"
                     % (4 * len(ov), 8 * K * K, 4 * len(ov)))
            kname += " + tree64 + map finalize"
        else:
            bpu, bnote = 4 * len(ov), "the request's input only: the engine is latency-bound (DESIGN.md 4)"
        workload = ("e_step of demo1's structure, 6 states, A1 B1 and the hidden parent D1 observed, "
                    "B=%d seq/GPU x T=%d (%s)" % (B, T, kname))
        metric = "sequence-timesteps/s batched e_step, demo1 with its hidden parent observed"
    elif name in ("estep_opchain_wide", "estep_opchain_wide_jt"):
        if kname.startswith("op_wide_msgs_kernel"):
            NP = 32 if N <= 32 else 64
            bpu = 2 * 4 * len(ov) + 4 * 8 * NP + 8
            bnote = ("obs %d (read by the filters and op_wide_xi_kernel) + alpha^ and beta^ written and read back "
                     "(4 x %d) + the forward scale exponent written and read 8; the xi sums are slab rows "
                     "(one per 16 sequences), the operators L2 / MALL reads" % (2 * 4 * len(ov), 8 * NP))
            kname += " + tree64 + map finalize"
        else:
            bpu, bnote = 4 * len(ov), "the request's input only: the engine is latency-bound (DESIGN.md 4)"
        workload = ("e_step of demo1's structure, 20 states, A1 B1 and the hidden parent D1 observed (9261 "
                    "evidence combinations), B=%d seq/GPU x T=%d (%s)" % (B, T, kname))
        metric = "sequence-timesteps/s batched e_step, demo1 @ 20 with its hidden parent observed"
    elif name == "em":
        kname += " + tree64 + finalize"
        workload = ("config4: em_learn iterations of HMM-shaped DBN, %d hidden x %d observed, "
                    "B=%d seq/GPU x T=%d, %d GPU(s), %s" % (
                        N, M, B, T, world,
                        "one packed RCCL all-gather per iteration" if world > 1 else
                        "no collective at world 1 (the packed RCCL all-gather runs at N > 1)"))
        metric = "sequence-timesteps/s em_learn (E-step + exchange + M-step per iteration), 16-state DBN"
        P = model.partial_size()
        extra["em"] = {"iterations_timed": steps, "ll_per_iteration": em_state["ll"][-steps:],
                       "exchange_ms_median": float(np.median(em_state["exchange_ms"][-steps:])),
                       "exchange_bytes_per_rank": 8 * (P + 2),
                       "note": ("kernel_ms is the whole iteration on the launch stream (the e_step kernel "
                                "(%s), the slab trees, exchange, finalize, host m_step); the exchange packs "
                                "the e_step partial (%d doubles incl. its 3-slot route tag), the ll tree sum "
                                "and the failure count" % (kname.split(" + ")[0], P))}
    elif name == "generate":
        bpu, bnote = 4 * model.num_vars, "the int32 draws written; the tables stay in cache"
        workload = "generate_data: HMM-shaped DBN, %d hidden x %d observed states, B=%d series/GPU x T=%d" % (
            N, M, B, T)
        metric = "sequence-timesteps/s generate_data (sampling), 16-state DBN"
    elif name == "jtree":
        bpu, bnote = 4 + 8 * N, "the request's I/O only: the engine is latency-bound (DESIGN.md 4)"
        workload = ("general join-tree engine: factorial HMM, X and Y 4 states each, O1 16 states of both, "
                    "X1 posterior, B=%d seq/GPU x T=%d" % (B, T))
        metric = "sequence-timesteps/s fwd-bwd smoothing, factorial HMM (general join-tree engine)"
    elif name in ("opchain_wide", "opchain_wide_jt"):
        if kname.startswith("op_wide_msgs_kernel"):
            NP = 32 if N <= 32 else 64
            bpu, bnote = 4 * len(ov) + 4 * 8 * NP + 8 * N, (
                "obs %d + alpha^ and beta^ written and read back (4 x %d) + the joint posterior %d (the "
                "operators are L2 / MALL reads)" % (4 * len(ov), 8 * NP, 8 * N))
        else:
            bpu, bnote = 4 * len(ov) + 8 * N, "the request's I/O only: the engine is latency-bound (DESIGN.md 4)"
        workload = ("demo1 structure, 20 states, A1 B1 and the hidden parent D1 observed, C1 posterior, "
                    "B=%d seq/GPU x T=%d (%s)" % (B, T, kname))
        metric = "sequence-timesteps/s fwd-bwd smoothing, demo1 @ 20 with its hidden parent observed"
    elif name in ("opchain", "opchain_jt"):
        if kname == "op_fb_kernel":
            bpu, bnote = 4 * len(ov) + 2 * 128 + 8 * N, (
                "obs %d + the 16-wide interface message written and read back (128 + 128) + posterior %d"
                % (4 * len(ov), 8 * N))
        else:
            bpu, bnote = 4 * len(ov) + 8 * N, "the request's I/O only: the engine is latency-bound (DESIGN.md 4)"
        workload = ("demo1 structure, 6 states, A1 B1 and the hidden parent D1 observed, C1 posterior, "
                    "B=%d seq/GPU x T=%d (%s)" % (B, T, kname))
        metric = "sequence-timesteps/s fwd-bwd smoothing, demo1 with its hidden parent observed"
    elif name == "joint":
        K = 16                         # joint interface states (X1, Y1)
        if kname == "chain_fb_ckpt_kernel<proj>":
            # X1's marginal written by the chain kernel itself (chain_ckpt.hip norm_store)
            ck = 8 * K // 4
            bpu, bnote = 4 * len(ov) + 2 * ck + 8 * N, (
                "obs %d + every 4th joint message as a checkpoint (%d written + %d read) + X1's marginal %d, "
                "written by the chain kernel (the joint posterior stays on chip)" % (4 * len(ov), ck, ck, 8 * N))
        else:
            kb, _ = kernel_bytes(kname, K, len(ov), True)
            bpu, bnote = kb + 8 * K + 8 * N, ("the chain kernel's bytes at K = 16 joint states, then the "
                                              "projection: the joint posterior read back, X1's marginal written")
            kname += " + project_kernel"
        workload = ("joint-interface chain: factorial HMM, X and Y 4 states each, O1 16 states of both, "
                    "X1 posterior, B=%d seq/GPU x T=%d" % (B, T))
        metric = "sequence-timesteps/s fwd-bwd smoothing, factorial HMM (joint-interface chain kernels)"
    elif name == "config3":
        workload = "config3: demo1.net structure, 5 vars x 32 states, A1 B1 observed, C1 posterior, " \
                   "B=%d seq/GPU x T=%d" % (B, T)
        metric = "sequence-timesteps/s fwd-bwd smoothing, demo1 @ 32 states"
    else:
        workload = "config5: wide clique {X0,Y1,Z1,X1} 64^4 entries, O1 16 states observed, X1 posterior, " \
                   "B=%d seq/GPU x T=%d; the 16.7M-entry in-clique is marginalised once per model version on " \
                   "the GPU (fold_lane_kernel, the line's fold field) and the timed step is the folded " \
                   "64-state chain" % (B, T)
        metric = "sequence-timesteps/s fwd-bwd smoothing, wide-clique DBN (64^4 in-clique)"
    achieved = bpu * B * T / (kern_ms * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": load_traffic(workload, name in ("fb", "config3", "config5", "joint", "opchain")),
            "kernel": kname,
            "kernel_ms": kern_ms, "bytes_per_unit": bpu, "bytes_note": bnote}
    if cfg in PRIMARY_BYTES and name in ("fb", "config3", "em", "estep", "config5"):
        pb = PRIMARY_BYTES[cfg]
        rate = pb * B * T / (kern_ms * 1e-3) / 1e9
        roof["primary"] = {"bytes_per_unit": pb, "equivalent_gbs": rate, "frac": rate / HBM_PEAK_GBS,
                           "note": "SURVEY 8(d)'s per-unit figure at this kernel time: a like-for-like "
                                   "comparison, not bandwidth the chip delivered"}
    base = kname.split(" + ")[0]
    if base in LATENCY_STEP:
        cyc, spb, bpc = LATENCY_STEP[base]
        rounds = -(-((B + spb - 1) // spb) // (N_CU * bpc))
        floor_ms = rounds * T * cyc / (CLOCK_GHZ * 1e9) * 1e3
        roof["latency"] = {"bound": "filter dependency chain", "cycles_per_step": cyc, "steps": T,
                           "block_rounds": rounds, "clock_ghz": CLOCK_GHZ, "floor_ms": floor_ms,
                           "frac": floor_ms / kern_ms,
                           "source": "profiles/r06/gpu/r06a_mb_lat6.txt (V4, the 16-state step) and "
                                     "profiles/r03/r03x_mb_lat.txt (V3, the 32-state step)"}
        if spb == 16:
            # round 6: the other forms of the 16-state step
            roof["latency"]["step_forms"] = {
                "V4 chained (the kernels)": 424, "V5 4 K-slices + add tree": 468,
                "V6 2 x 2-MFMA chains + add": 444, "V7 4 K-slices, evidence in the tree": 416,
                "note": "no form is more than 2% shorter than the chained step, so the chained step's "
                        "424 cycles set the ceiling (DESIGN.md 5)"}
    pr = pipe_roof(workload, kern_ms)
    if pr:
        roof["pipe"] = pr
    if base == "chain_row64_kernel":
        ir = row64_issue_roof(B, T, kern_ms)
        if ir:
            roof["issue"] = ir
    rec = {"metric": metric, "value": value, "unit": "sequence-timesteps/s", "n_gpus": world,
           "steps": steps, "warmup": nw, "warmup_requested": warmup, "ms_per_step": elapsed / steps * 1e3,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
           "data": "synthetic",
           "config": {"workload": workload, "B_per_gpu": B, "T": T, "hidden_states": N,
                      "observed_states": M, "observed_vars": len(ov), "parallelism": "dp%d" % world},
           "roofline": roof}
    rec.update(extra)
    if rank == 0 and world == 1 and name in ("fb", "config3", "config5") and headline:
        # PCIe-inclusive figure: the same batch from host buffers
        # through nipamd_fb_host (H2D obs, kernels, D2H posteriors)
        host_obs = np.ascontiguousarray(obs_np)
        nip_amd.forward_backward_inference_host(model, host_obs, ov, [q])
        t1 = time.perf_counter()
        nip_amd.forward_backward_inference_host(model, host_obs, ov, [q])
        el1 = time.perf_counter() - t1
        rec["pcie_inclusive"] = {"value": B * T / el1, "unit": "sequence-timesteps/s", "ms": el1 * 1e3,
                                 "note": "host buffers in and out (pageable), one call; not the headline"}
    if name == "config5":
        # the in-clique marginalisation: 64^4 entries summed over the hidden
        # parents on the GPU (fold.hip), once per model version
        fms, fby = [], 0.0
        for _ in range(5):
            _, ms_f, fby = model.fold()
            fms.append(ms_f)
        fk = float(np.median(fms))
        rec["fold"] = {"kernel": "fold_lane_kernel + fold_sum_kernel", "kernel_ms": fk, "bytes": fby,
                       "roofline": {"bound": "hbm", "achieved": fby / (fk * 1e-3) / 1e9,
                                    "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                    "frac": fby / (fk * 1e-3) / 1e9 / HBM_PEAK_GBS},
                       "note": "A[x][y] = sum over Y1, Z1 of the 134 MB clique x priors, per model version"}
    del obs, ll, st
    torch.cuda.empty_cache()
    return rec


# The printed line must fit the driver's ~8 KB stdout tail with every config
# in it (config 3 fell off a 14 KB line): each record keeps its
# figures -- ms_per_step, value, roofline frac / achieved / traffic, the other
# roofs' frac and floor -- and the long notes, byte breakdowns and sources go
# to the detail file (--detail, default gpurun_out/bench_detail.json).
ROOF_KEEP = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_ms", "bytes_per_unit")


def compact_roof(roof):
    r = {k: roof[k] for k in ROOF_KEEP if k in roof}
    for k in ("primary", "latency", "pipe", "issue"):
        if k in roof:
            r[k] = {"frac": roof[k]["frac"]}
            if "floor_ms" in roof[k]:
                r[k]["floor_ms"] = roof[k]["floor_ms"]
            if k == "issue" and "at_4_cycles" in roof[k]:
                r[k]["frac_at_4cyc"] = roof[k]["at_4_cycles"]["frac"]
            if k == "issue" and "measured_step_cycles" in roof[k]:
                m = roof[k]["measured_step_cycles"]
                r[k]["step_cycles"] = {"alone": m["alone_fwd"], "in_kernel": m["in_kernel"]}
    return r


def compact_cpu(cb):
    if not cb or "value" not in cb:
        return cb
    r = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample") if k in cb}
    if "port" in cb:
        r["port_value"] = cb["port"]["value"]
    return r


def compact(rec, secondary=False):
    if secondary:
        r = {k: rec[k] for k in ("value", "ms_per_step", "steps", "warmup") if k in rec}
        r["workload"] = rec["config"]["workload"]
    else:
        r = {k: v for k, v in rec.items() if k not in ("roofline", "cpu_baseline", "secondary", "em", "fold")}
    r["roofline"] = compact_roof(rec["roofline"])
    if "cpu_baseline" in rec:
        r["cpu_baseline"] = compact_cpu(rec["cpu_baseline"])
    if "em" in rec:
        r["em"] = {k: rec["em"][k] for k in ("exchange_ms_median", "exchange_bytes_per_rank")}
    if "fold" in rec:
        r["fold"] = {"kernel_ms": rec["fold"]["kernel_ms"], "frac": rec["fold"]["roofline"]["frac"]}
    if "pcie_inclusive" in rec:
        r["pcie_inclusive"] = {k: rec["pcie_inclusive"][k] for k in ("value", "ms")}
    return r


def rounded(x):
    """Floats to 6 significant digits (the line's size; the detail file keeps all)."""
    if isinstance(x, float):
        return float("%.6g" % x)
    if isinstance(x, dict):
        return {k: rounded(v) for k, v in x.items()}
    if isinstance(x, list):
        return [rounded(v) for v in x]
    return x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=0, help="timed steps of the headline (0: the workload's)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0, help="sequences per GPU (0: the workload's)")
    ap.add_argument("--T", type=int, default=0, help="time slices (0: the workload's)")
    ap.add_argument("--N", type=int, default=16)
    ap.add_argument("--M", type=int, default=16)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="fb",
                    help="fb: the headline metric (config 2 smoothing) plus the secondary configs; "
                         "estep: one batched e_step (config 4 per-GPU shard); em: config 4, one step = "
                         "one em_learn iteration (m_step, e_step of the shard, the packed all-gather "
                         "over RCCL, finalize); config3: demo1 @ 32 states smoothing; config5: wide-"
                         "clique smoothing; jtree: a factorial HMM on the general join-tree engine; "
                         "joint: the same slice as a joint-interface chain; generate: generate_data")
    ap.add_argument("--no-secondary", action="store_true", help="the headline workload only")
    ap.add_argument("--min-warm", type=float, default=0.5,
                    help="after the W warmup steps, add untimed steps (at most 64) until this many seconds "
                         "of warmup ran, as the secondary lines do: the f64 kernels run their first "
                         "launches at a lower clock (config 2: 0.278-0.288 ms per step after 3 warmup "
                         "steps, 0.243-0.252 after 0.5 s, profiles/r05/gpu/r05av_warm.txt); 0 = exactly W. "
                         "The line's 'warmup' is the count that ran, 'warmup_requested' W")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=8.0, help="seconds per CPU baseline")
    ap.add_argument("--no-check", action="store_true", help="skip the output sanity check (ablation builds)")
    ap.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="the full records (notes, byte breakdowns, roof sources) as JSON ('' = none)")
    args = ap.parse_args()
    world = launch_or_check(args, sys.argv[1:])
    rank = int(os.environ.get("RANK", "0"))
    secondary = [] if (args.no_secondary or args.workload != "fb" or args.batch or args.T) else SECONDARY

    # CPU baselines first, in a child process, while nothing here has touched the GPU
    cpu = {}
    if world == 1 and rank == 0 and not args.no_cpu_baseline and args.workload != "generate":
        cpu = cpu_baselines([args.workload] + secondary, args.cpu_budget)

    import torch
    import torch.distributed as dist

    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    steps = args.steps or WORKLOADS[args.workload][6]
    rec = run_workload(args.workload, args, world, rank, dev, steps, args.warmup, min_warm_s=args.min_warm)
    if args.workload in cpu:
        rec["cpu_baseline"] = cpu[args.workload]
    if world == 1 and rank == 0 and not args.no_cpu_baseline and args.workload == "generate":
        rec["cpu_baseline"] = cpu_baseline_generate(*WORKLOADS["generate"][1](args), T=rec["config"]["T"])
    line = compact(rec)
    detail = {"headline": rec}
    if secondary:
        sec, full = {}, {}
        for w in secondary:
            r = run_workload(w, args, world, rank, dev, WORKLOADS[w][6], 2 if w != "em" else 1, min_warm_s=0.5)
            if w in cpu:
                r["cpu_baseline"] = cpu[w]
            key = WORKLOADS[w][0] if w != "estep_config3" else "config3_estep"
            full[key] = r
            sec[key] = compact(r, secondary=True)
        line["secondary"] = sec
        detail["secondary"] = full
    if rank == 0:
        if args.detail:
            try:
                os.makedirs(os.path.dirname(os.path.abspath(args.detail)), exist_ok=True)
                with open(args.detail, "w") as f:
                    json.dump(detail, f, indent=1)
            except OSError as e:
                print("bench: detail file not written: %s" % e, file=sys.stderr)
        print(json.dumps(rounded(line)))
    if world > 1:
        dist.destroy_process_group()


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


if __name__ == "__main__":
    main()
