"""The MI355X training step: native kernels end to end, no autograd.

Per iteration (reference ``train.py:48-105``, intended semantics; all buffers time-major
(T, B, N, ...) so the first T steps of a rollout are one contiguous block):

rollout, t = 0.. (stops when every env is done; per-env done masks)
    scan(s_t)      -> kNN idx, TTC danger bits + counts, all-pairs safety of s_t
    ctrl_fwd(s_t)  -> a_t, s_{t+1}, pooled features + argmax slots (saved for backward),
                      per-env goal distance / action-loss sums
losses
    counts all-reduced over DP ranks (global pooled normalisation)
backward
    cbf_bwd (fused) -> h(s_t), h'(s_{t+1}) on the same slots, loss sums, dL/dh, dL/dh' formed
                      in-kernel, dL/d(s_i - s_j) per edge (h and h' paths) + CBF dW slabs
    rev_csr + node_reduce -> direct dL/ds_t (edge -> node, deterministic, no atomics)
    for t = T-1..0 (BPTT):  ctrl_node_bwd (its prologue forms G_{t+1} from step t+1's records:
                      the fused BPTT combine) -> ctrl_edge_bwd
                      (dA_t = dt*G_{t+1}[v] + action-loss grad; G_t = dL/ds_t)
    slab reductions -> the flat gradient buffer (then RCCL all-reduce + fused Adam).
"""
from __future__ import annotations

import os

import torch

from .. import config as C
from .. import knobs
from ..ops import layout as L
from ..ops import native
from ..ops.weights import PackedWeights


# action-loss weight of the total loss (core.py:174-184 via train.py:93,98); the node backward
# divides it by the all-reduced action count on the device
ACT_COEF = C.LOSS_SCALE * C.LOSS_WEIGHTS[4]
STEP_ROWS_BYTES = 64 << 20      # per-step slab rows for BPTT grids whose T x rows fit this (HipEngine.step_rows)
STATS_COLS = 18       # StepStats row: 10 loss sums | 3 counts | 3 local | skipped | loss scale
STATS_RING = 256


class HipEngine:
    name = "hip"
    resort_every = 4          # scan: Hilbert re-sort period (rollout steps)
    overlap_hfwd = False      # CBF h of the main slots on a side stream during the rollout. Off: the
                              # one-launch controller steps hold a CU's LDS (145 KB) and the 1024-thread
                              # scan blocks leave no room either, so the slices only delay the rollout's
                              # critical chain (A/B fp32 15.04 vs 14.60 ms, bf16 8.06 vs 7.92 ms; round 1,
                              # with smaller scan blocks, measured the overlap 7.83 -> 7.63 ms for bf16)
    native_rollout = True     # per-step launch loop in C++ (csrc/runtime.cpp)
    bptt_groups = 1           # independent env groups whose BPTT chains run on separate streams
    native_bptt = True        # reverse-time BPTT launch loop in C++ (csrc/runtime.cpp)
    check_every = 0           # early-stop host check period of the native driver (0: auto -- every
                              # step at >= 16K agents per rank, up to every 4th for small scenes)
    reduce_late = 0           # >0: dS steps reduced before the BPTT starts, the rest on the aux stream
                              # during it (A/B on MI355X: neutral-to-slower, 7.63 vs 7.66 ms; off)
    small_rollout = True      # envs of <= native.SMALL_MAXN graph nodes: the whole rollout is ONE
                              # persistent launch (one workgroup per env, device-side early stop)
    bwd_graph = True          # small scenes (the persistent rollout's <= 64-node envs): everything after
                              # the rollout (counts, CBF losses + backward, BPTT, gradient assembly)
                              # replayed from a HIP graph captured once per horizon T -- the host issues
                              # ~30 launches there and the GPU waited for it (config #2: ~0.1 ms of host
                              # gaps per iteration, profiles/r5_b2/)

    def __init__(self, trainer):
        self.tr = trainer
        cfg = trainer.cfg
        # scheduling choices are class attributes (tests / A/B scripts set them); the environment
        # knobs that remain are listed in macbf_gnn_amd/knobs.py
        # instance snapshots of the class-level choices (a test may reset the class attribute)
        self.bptt_groups = int(self.bptt_groups) if cfg.num_envs % self.bptt_groups == 0 else 1
        self._drv = None
        self._bdrv = None
        self.native_bptt = bool(knobs.get_int("MACBF_NATIVE_BPTT", int(self.native_bptt)))
        self.bptt = cfg.bptt
        self.reuse = cfg.reuse_nbr_idx
        # deduplicated h/h' evaluations need both roles' state gradients on the same s_t: BPTT only
        self.dedup = bool(getattr(cfg, "cbf_dedup", True)) and cfg.bptt
        native.lib()
        self.dev = trainer.device
        self.B, self.N = cfg.num_envs, cfg.num_agents
        self.D = cfg.dim
        self.W = native.rec_width(self.D)
        self.M = cfg.num_obstacles * cfg.obstacle_points          # static obstacle nodes per env
        self.Nn = self.N + self.M
        self.K = min(self.Nn, cfg.top_k)
        if self.K > C.MAX_TOP_K:
            raise ValueError(f"top_k <= {C.MAX_TOP_K} supported by the native kernels")
        self.Tmax = cfg.inner_loops
        self.small_rollout = self.small_rollout and self.native_rollout and self.Nn <= native.SMALL_MAXN
        ov = knobs.get_int("MACBF_OVERLAP_HFWD", -1)
        if ov >= 0:
            self.overlap_hfwd = bool(ov)
        elif cfg.dtype == "fp32" and 12288 <= self.B * self.N <= 24576:
            # the 16-env per-rank work of config #3 at DP 4 (16,384 agents): the h slices fill CUs the
            # controller step leaves idle -- 3.987-3.998 vs 4.044-4.076 ms interleaved; at 8 envs
            # neutral (2.806-2.862 vs 2.821-2.870), at 32 envs slower (6.55-6.58 vs 6.25),
            # profiles/r6_runs/r6ar/, r6as/
            self.overlap_hfwd = True
        if self.small_rollout:
            self.overlap_hfwd = False     # the CBF h of all main slots runs after the one-launch rollout
        # kernel precision (csrc/prec.h): bf16 / fp16 MFMA inputs, or "fp32" -- the reference
        # precision, fp32-accurate 3-term split-bf16 kernels (x3)
        mdt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}.get(cfg.dtype)
        if mdt is None:
            raise ValueError(f"dtype must be bf16, fp16 or fp32 on the HIP path, got {cfg.dtype!r}")
        self.pw = PackedWeights(trainer.fp, self.D, mdt)
        self.prec = self.pw.prec
        self.hdt = self.pw.dtype                 # packed / pooled element type (bf16 | fp16)
        self.prow = L.pooled_row(self.prec)      # pooled / dL/dpooled row: [hi | lo] for fp32
        offs = {pn: o for (m, pn, shape, o, n) in trainer.fp.specs}
        self._alloc()
        node_map = L.ctrl_node16_grad_map if self.node16_w is not None else L.ctrl_node_grad_map
        # flat-gradient assembly: CSR (by parameter) over the concatenated reduced slabs
        # [cbf | node | edge]; one gather launch per iteration (deterministic)
        import numpy as np
        srcs, dsts, base = [], [], 0
        for name, fn, width in (("cbf", L.cbf_grad_map, native.CBF_PARTIAL),
                                ("node", node_map, native.CTRL_NODE_PARTIAL),
                                ("edge", L.ctrl_edge_grad_map, native.CTRL_EDGE_PARTIAL)):
            sm, dm = fn(offs, self.D)
            sm, dm = np.asarray(sm, dtype=np.int64), np.asarray(dm, dtype=np.int64)
            if sm.size and (sm.min() < 0 or sm.max() >= width or dm.min() < 0 or dm.max() >= trainer.fp.numel):
                raise ValueError(f"gradient map {name} out of range")
            srcs.append(sm + base)
            dsts.append(dm)
            base += width
        srcs, dsts = np.concatenate(srcs), np.concatenate(dsts)
        order = np.lexsort((srcs, dsts))
        counts = np.bincount(dsts, minlength=trainer.fp.numel)
        gptr = np.concatenate([[0], np.cumsum(counts)])
        mk32 = lambda a: torch.as_tensor(a, dtype=torch.int32, device=self.dev)
        self.g_ptr, self.g_src = mk32(gptr), mk32(srcs[order])
        # DP: the CBF range of the flat gradient is final once the CBF slabs are reduced, before the
        # BPTT starts; its all-reduce is issued then (async) and joined before Adam, so at world > 1
        # it is in flight during the BPTT. The controller range is
        # all-reduced after the BPTT. Both ranges are contiguous in the flat buffer.
        rng = {}
        for m, pn, shape, o, n in trainer.fp.specs:
            lo, hi = rng.get(m, (o, o))
            rng[m] = (min(lo, o), max(hi, o + n))
        if sum(hi - lo for lo, hi in rng.values()) != trainer.fp.numel or set(rng) != {"controller", "cbf"}:
            raise ValueError("flat parameters must be the contiguous controller and CBF ranges")
        self.grad_ranges = rng
        self._grad_work = None
        # whole-iteration HIP graph (cfg.graph): rollout to Tmax with device-side done masks,
        # losses, backward; replayed per iteration (removes the per-kernel launch / Python cost
        # that dominates small configurations). Sampling, the DP all-reduces and the optimizer
        # stay eager around the two captured graphs.
        self.graph_mode = bool(getattr(cfg, "graph", False))
        self._graphs = None
        self._graph_gs = None
        # (per-T backward graphs for every scene size, not only small ones: headline 10.125-10.135
        # vs 10.141-10.165 ms, 8-env slice 2.798-2.803 vs 2.793-2.815 -- within noise, profiles/r6d/)
        self.bwd_graph = bool(knobs.get_int("MACBF_BWD_GRAPH", int(self.bwd_graph)))
        self._bwd_graphs = {}          # (T, grad scale) -> CUDAGraph of _counts + _backward
        self._graph_table = None       # key suffix of the graphs registered with the rollout driver
        self._scenario = None          # (s0, g) the next small-scene rollout loads itself
        self._kernel_scenario = bool(knobs.get_int("MACBF_KERNEL_SCENARIO", 1))
        self._graph_launch = False     # the next run_small launches the registered graph of its T
        self._launched_T = None
        self._drv_launch = bool(knobs.get_int("MACBF_GRAPH_LAUNCH", 1))
        self._bwd_pool = None
        self._bwd_capture = False
        # int32 guard flag the gradient-assembly launch clears on a non-finite element (set by the
        # trainer for single-process runs; with DP the check follows the all-reduce)
        self.check_ok = None
        # the 16x16x32 backward kernels this engine runs, once before training (ops/selfcheck.py: a
        # miscompiled schedule stops here instead of corrupting gradients): CBF / edge against their
        # float64 oracles (x3), the node kernel against the 32x32x16 one (every precision)
        self.selfcheck = None
        from ..ops import selfcheck
        if selfcheck.enabled():
            self.selfcheck = selfcheck.check(self)

    # ------------------------------------------------------------------ buffers
    def _alloc(self):
        B, N, K, T, dev = self.B, self.N, self.K, self.Tmax, self.dev
        D, W, Nn = self.D, self.W, self.Nn
        f32, i32, u8, bf = torch.float32, torch.int32, torch.uint8, self.hdt
        # node records (agents, then static obstacle points), time-major
        self.S = torch.zeros(T + 1, B, Nn, W, dtype=f32, device=dev)
        self.G = torch.zeros(B, N, D, dtype=f32, device=dev)
        self.A = torch.zeros(T, B, N, D, dtype=f32, device=dev)
        # one extra graph when h' uses the recomputed kNN of s_{t+1} (reuse_nbr_idx=False)
        G1 = 0 if self.reuse else 1
        self.idx = torch.zeros(T + G1, B, N, K, dtype=i32, device=dev)
        self.dang = torch.zeros(T, B, N, K, dtype=u8, device=dev)
        self.cnt = torch.zeros(T, B, 2, dtype=f32, device=dev)
        self.safe = torch.zeros(T + 1, B, dtype=f32, device=dev)
        # per-env goal-distance / action-term sums, fixed point (native.FX_*): order-independent
        self.dist = torch.zeros(T, B, dtype=torch.int64, device=dev)
        self.act = torch.zeros(T, B, dtype=torch.int64, device=dev)
        self.pooled = torch.zeros(T, B, N, self.prow, dtype=bf, device=dev)
        self.argmax = torch.zeros(T, B, N, 128, dtype=u8, device=dev)
        self.dE = torch.zeros(2 * T * B * N * K * W, dtype=f32, device=dev)
        self.rptr = torch.zeros((T + G1) * B, Nn + 1, dtype=i32, device=dev)
        self.redges = torch.zeros((T + G1) * B, N * K, dtype=i32, device=dev)
        self.dS = torch.zeros(T + 1, B, N, W, dtype=f32, device=dev)
        self.Gb = torch.zeros(T + 1, B, N, W, dtype=f32, device=dev)
        self.dP = torch.zeros(B, N, self.prow, dtype=bf, device=dev)
        self.ego = torch.zeros(B, N, W, dtype=f32, device=dev)
        # per-edge controller records of the BPTT, double-buffered by step parity: step t's edge
        # backward writes dEc[t & 1] while the node backward of step t forms G_{t+1} from
        # dEc[(t+1) & 1] (in-edges of agents of other workgroups: in the fused node+edge launch the
        # two phases of different workgroups overlap)
        self.dEc = torch.zeros(2, B, N, K, W, dtype=f32, device=dev)
        self.counts = torch.zeros(3, dtype=f32, device=dev)
        self.local = torch.zeros(3, dtype=f32, device=dev)        # agent-steps, safe agents, action-loss sum
        self.raw_stats = torch.zeros(STATS_COLS, dtype=f32, device=dev)   # graph mode (fixed address)
        self._stats_pending = None
        # per-iteration statistics rows (utils.metrics.StepStats layout), written by one kernel per
        # iteration into a ring; a full ring is replaced by a fresh one (torch.empty: no kernel), so
        # a StepStats keeps its row for as long as it is referenced
        self._ring = torch.empty(STATS_RING, STATS_COLS, dtype=f32, device=dev)
        self._ring_pos = 0
        # cnt / safe / dist / act are accumulated by atomics: rollout_stats zeroes them after reading
        # (no fill kernels in the training step); a rollout not followed by _counts zeroes them first
        self._sums_dirty = False
        self.valid_buf = torch.zeros(T, B, dtype=u8, device=dev)
        # exploration noise (reference train.py:65-67): counter-based device RNG keyed per iteration
        self.noise_key = torch.zeros(1, dtype=torch.int64, device=dev)
        # persistent rollout: [envs done, max step, finished workgroups] (re-armed by the kernel)
        self.small_ctl = torch.zeros(3, dtype=i32, device=dev)
        self.small_stamps = None          # diagnostics: [env][wave][16] phase clocks of the persistent rollout
        # K = 12, x3: the 16x16x32 controller edge backward (csrc/ctrl16.h, 8-wave workgroups); the
        # 1-pass builds keep the 32x32x16 kernel (70 vs 78 us per call in bf16, 74 vs 89 us fp16 3-D,
        # profiles/r4_validate/). MACBF_EB16=0/1 forces either. Decided before the grids (per-CU residency)
        self.eb16_w = (self.pw.ctrl_w16 if (K == 12 and knobs.get_int("MACBF_EB16", int(self.prec == "fp32")))
                       else None)
        eb16 = self.eb16_w is not None
        self.nb_node, self.nb_edge = native.ctrl_bwd_grids(B * N, dev, self.prec, eb16=eb16)
        # BPTT env groups (independent chains on separate streams): per-group grids and slab rows
        Gp = self.bptt_groups
        if Gp < 1 or B % Gp:
            raise ValueError(f"bptt_groups={Gp} must divide num_envs={B}")
        self.grp_nb = native.ctrl_bwd_grids((B // Gp) * N, dev, self.prec, eb16=eb16)
        # slab rows each BPTT path writes (and the slab reduction reads): exactly those, so rows no
        # path writes are never summed
        self.slab_rows = (self.nb_node, self.nb_edge) if Gp == 1 else (Gp * self.grp_nb[0], Gp * self.grp_nb[1])
        # small grids (config #2: one node and 16 edge workgroups): every reverse step writes its own
        # slab rows (no read-modify-write of the previous step's partial at each kernel's end) and
        # the tail reduction sums T x rows -- at most a few MB; large grids keep one accumulated row
        # per workgroup (T x 256 rows would cost the reduction more than the RMW costs the chain)
        self.step_rows = bool(Gp == 1 and self.bptt and
                              T * (self.nb_node * native.CTRL_NODE_PARTIAL + self.nb_edge * native.CTRL_EDGE_PARTIAL) * 4
                              <= STEP_ROWS_BYTES)
        # small scenes: the persistent rollout keeps the node MLP's activations for the cooperative
        # (32-agent chunk) node backward, which then skips its L1..L4 recompute (native drivers
        # only). Config #2 bf16 0.88-0.91 vs 0.97 ms; the 8-env slice (launch-per-step x3 path,
        # whose store-keeping step kernel spills) 2.87 vs 2.78-2.83 ms: off there (docs/PERF.md)
        self.node_acts = None
        self._acts_valid = False
        if (self.bptt and self.small_rollout and native.node_bwd_chunk(B * N, dev) == 32
                and knobs.get_int("MACBF_NODE_ACTS", 1)):
            self.node_acts = torch.empty(T * B * N * native.node_act_bytes(self.prec), dtype=torch.uint8, device=dev)
        rows_n, rows_e = self.slab_rows
        if self.step_rows:
            rows_n, rows_e = T * rows_n, T * rows_e
        self.part_node = torch.zeros(max(rows_n, B), native.CTRL_NODE_PARTIAL, dtype=f32, device=dev)
        self.part_edge = torch.zeros(max(rows_e, B), native.CTRL_EDGE_PARTIAL, dtype=f32, device=dev)
        self.gstreams = [torch.cuda.Stream(device=dev) for _ in range(Gp - 1)]
        self.red_all = torch.zeros(native.CBF_PARTIAL + native.CTRL_NODE_PARTIAL + native.CTRL_EDGE_PARTIAL,
                                   dtype=f32, device=dev)
        self.red_cbf, self.red_node, self.red_edge = torch.split(
            self.red_all, [native.CBF_PARTIAL, native.CTRL_NODE_PARTIAL, native.CTRL_EDGE_PARTIAL])
        if self.dedup:
            E = T * B * N * K
            self.map1 = torch.zeros(T, B, N, K, dtype=i32, device=dev)
            self.src = torch.zeros(2 * E, dtype=i32, device=dev)
            self.mcnt = torch.zeros(T * B * N, dtype=i32, device=dev)
            self.hbuf = torch.zeros(2 * E, dtype=f32, device=dev)
            self.hmask = torch.zeros(2 * E, dtype=u8, device=dev)
            self.dhbuf = torch.zeros(2 * E, dtype=f32, device=dev)
            ndh = native.cbf_dh_grid(2 * E, dev)
            self.loss_part = torch.zeros(ndh, native.DH_PARTIAL, dtype=f32, device=dev)
            self.blk_active = torch.zeros(ndh, dtype=i32, device=dev)
            # x3: the 16x16x32 backward (csrc/cbf16.h, two waves per SIMD) reads cbf_compact's
            # 16-byte records of the active evaluations; bf16 / fp16: the 32x32x16 kernel on the
            # index list (already two waves per SIMD there; 1635 vs 1791 us per call in bf16,
            # profiles/r4_validate/)
            self.cbf16 = self.prec == "fp32"
            self.act_list = torch.zeros(2 * E, dtype=i32, device=dev) if not self.cbf16 else None
            self.rec_list = torch.zeros(2 * E, 4, dtype=i32, device=dev) if self.cbf16 else None
            self.loss_red = torch.zeros(native.DH_PARTIAL, dtype=f32, device=dev)
            self.nev_host = torch.zeros(1, dtype=i32, device=dev)     # unused by host-range slices
            self.nev_dev = torch.zeros(1, dtype=i32, device=dev)      # [U] of the match
            self.nact_dev = torch.zeros(1, dtype=i32, device=dev)     # active evaluations
            self.hstream = torch.cuda.Stream(device=dev)              # rollout-overlapped CBF h slices
        # 128-agent node chunks: the 16x16x32 node backward (csrc/node16.h, 8-wave workgroups; every
        # precision: 55 vs 59 us per call in bf16, 62 vs 66 us fp16 3-D, profiles/r4_validate/);
        # MACBF_NODE16=0: the 32x32x16 kernel (A/B runs). Decided once per engine (its slab layout
        # differs, layout.ctrl_node16_grad_map): the BPTT launches cover (B / groups) x N agents,
        # the no-BPTT launch T x B x N >= that, so every node launch of this engine takes the same kernel
        Gp = self.bptt_groups
        self.node16_w = (self.pw.node_rm16 if (knobs.get_int("MACBF_NODE16", 1)
                                               and native.node_bwd_chunk((B // Gp) * N, dev) == 128) else None)
        self.host_dist = torch.zeros(T, B, dtype=torch.int64, pin_memory=True)
        self.copy_stream = torch.cuda.Stream(device=dev)
        self.aux = torch.cuda.Stream(device=dev)      # reverse-CSR build overlaps the CBF kernel
        self._nobptt = {}     # lazily sized (T*B)-batched controller-backward buffers
        self._part_cbf = {}
        self._part_cbf_nb = {}

    def after_update(self, commit=None):
        self.pw.update(commit=commit)

    # ------------------------------------------------------------------ rollout
    def _noise_args(self):
        cfg = self.tr.cfg
        if cfg.add_noise_prob <= 0:
            return dict(noise_key=None)
        return dict(noise_key=self.noise_key, noise_prob=float(cfg.add_noise_prob), noise_scale=float(cfg.noise_scale))

    def load_inputs(self, s0, g, obs=None, defer=False):
        """Scenario -> the static input buffers (start records, goals, obstacle rows) and the
        exploration-noise key of this iteration (seed, iteration, rank). defer: the persistent
        small-scene rollout loads the start records and goals itself (self._scenario)."""
        if self.tr.cfg.add_noise_prob > 0:
            from ..ops.scenario import iteration_key
            self.noise_key.fill_(iteration_key(self.tr.cfg.seed, int(self.tr.step_count), self.tr.dp.rank, salt=0x4E4F4953))
        B, N, D = self.B, self.N, self.D
        self._scenario = None
        # (inputs the kernel cannot read as they are -- host tensors, other dtypes or layouts -- take
        # the copies below)
        defer = (defer and all(t.device == self.S.device and t.dtype == torch.float32 and t.is_contiguous()
                               for t in (s0, g))
                 and tuple(s0.shape) == (B, N, 2 * D) and tuple(g.shape) == (B, N, D))
        if defer:
            self._scenario = (s0, g)
        elif D == 2:
            self.S[0, :, :N].copy_(s0)
        else:
            # 3-D records (x, y, z, 0 | vx, vy, vz, 0): two strided copies into the record halves
            # (the pad lanes of S are zero from the allocation and never written)
            r = self.S[0, :, :N].view(B, N, 2, 4)
            r[..., 0, :3].copy_(s0[..., :3])
            r[..., 1, :3].copy_(s0[..., 3:6])
        if self.M:
            if obs is None or tuple(obs.shape) != (B, self.M, D):
                raise ValueError(f"expected obstacles of shape {(B, self.M, D)}")
            # static obstacle nodes in every time slice: one strided copy of the positions (their
            # velocity and pad lanes stay zero: no kernel writes them)
            self.S[:, :, N:, :D].copy_(obs.unsqueeze(0).expand(self.Tmax + 1, B, self.M, D))
        if not defer:
            self.G.copy_(g)
        return defer

    def rollout(self, s0, g, obs=None, early_stop=None):
        small = (self.small_rollout and self.native_rollout and not self.graph_mode and self._kernel_scenario
                 and not torch.cuda.is_current_stream_capturing())
        self.load_inputs(s0, g, obs, defer=small)
        return self._rollout_steps(self.tr.cfg.early_stop if early_stop is None else early_stop)

    def _driver(self):
        """The native rollout driver (csrc/runtime.cpp) over this engine's persistent buffers;
        every pointer it offsets per step is checked here once."""
        import os
        if self._drv is None:
            cfg = self.tr.cfg
            B, N, Nn, K, D, W, T = self.B, self.N, self.Nn, self.K, self.D, self.W, self.Tmax
            G1 = 0 if self.reuse else 1
            exp = {"S": (self.S, torch.float32, (T + 1, B, Nn, W)), "G": (self.G, torch.float32, (B, N, D)),
                   "A": (self.A, torch.float32, (T, B, N, D)), "idx": (self.idx, torch.int32, (T + G1, B, N, K)),
                   "dang": (self.dang, torch.uint8, (T, B, N, K)), "cnt": (self.cnt, torch.float32, (T, B, 2)),
                   "safe": (self.safe, torch.float32, (T + 1, B)), "dist": (self.dist, torch.int64, (T, B)),
                   "act": (self.act, torch.int64, (T, B)), "pooled": (self.pooled, self.hdt, (T, B, N, self.prow)),
                   "argmax": (self.argmax, torch.uint8, (T, B, N, 128))}
            for name, (t, dt, shape) in exp.items():
                native.check(t, dt, shape, name)
            if not self.host_dist.is_pinned() or tuple(self.host_dist.shape) != (T, B):
                raise native.NativeError("host_dist must be pinned (T, B)")
            pw = self.pw
            perm = native._perm_buf(B, Nn, self.dev)
            scan_f4 = native.scan_ws_f4(Nn)                          # large envs: global staging
            # owned by the engine (the driver keeps the pointer for its lifetime)
            self._scan_ws = torch.empty(max(B * scan_f4 * 16, 16), dtype=torch.uint8, device=self.dev)
            scan_ws = self._scan_ws if scan_f4 else None
            native._perm_sorted.add((B, Nn, str(self.dev)))      # sorted at t = 0 of every run
            overlap = bool(self.dedup and self.overlap_hfwd)
            BNK = B * N * K
            c = {k: native.ptr(v[0]) for k, v in exp.items()}
            c.update(dict(
                B=B, N=N, Nn=Nn, K=K, D=D, Tmax=T, num_cu=native.num_cu(self.dev), prec=L.PREC_CODE[self.prec],
                resort_every=int(self.resort_every), compute_safety=int(cfg.compute_safety), overlap_hfwd=int(overlap),
                hfwd_blocks=native.cbf_hfwd_grid(BNK, self.dev), L=float(max(1.0, N / C.AGENT_DENSITY) ** (1.0 / D)),
                perm=native.ptr(perm), host_dist=int(self.host_dist.data_ptr()),
                check_every=int(self.check_every or max(1, min(4, 16384 // (B * N)))),
                apw=int(native.ctrl_fwd_apw(B * N, self.dev, N)),
                ctrl_w=native.ptr(pw.ctrl_w), f_edge=int(pw.ctrl_off["ew1f"]), f_node=int(pw.ctrl_off["nw1f"]),
                ctrl_v=native.ptr(pw.ctrl_v), cbf_w=native.ptr(pw.cbf_w), f_fwd=int(pw.cbf_off["w1f"]),
                cbf_rm=native.ptr(pw.cbf_rm), cbf_v=native.ptr(pw.cbf_v),
                hbuf=native.ptr(self.hbuf) if overlap else 0, hmask=native.ptr(self.hmask) if overlap else 0,
                src=native.ptr(self.src) if overlap else 0, nev=native.ptr(self.nev_host) if overlap else 0,
                r2_train=float(C.DIST_MIN_THRES * C.DIST_MIN_THRES), ttc_train=float(C.TIME_TO_COLLISION),
                r2_check=float(C.DIST_MIN_CHECK * C.DIST_MIN_CHECK), ttc_check=float(C.TIME_TO_COLLISION_CHECK),
                dt=float(C.TIME_STEP), obs_r=float(C.OBS_RADIUS), sqrt3=float(C.SQRT3),
                dist_thr=float(C.DIST_MIN_THRES), dist_eps=float(C.CBF_DIST_EPS_COORD * D),
                done_thr=float(C.DIST_MIN_CHECK),
                noise_key=native.ptr(self.noise_key) if cfg.add_noise_prob > 0 else 0,
                scan_ws=native.ptr(scan_ws), scan_ws_env=int(scan_f4),
                small_ctl=native.ptr(self.small_ctl) if self.small_rollout else 0,
                small_apw=int(native.small_apw(N)), knn_tail=int(not self.reuse),
                small_stamps=native.ptr(self.small_stamps),     # diagnostics builds (scripts/stamps_small.py)
                node_acts=native.ptr(self.node_acts), node_act_bytes=native.node_act_bytes(self.prec),
                noise_prob=float(cfg.add_noise_prob), noise_scale=float(cfg.noise_scale),
                fork_device_scope=1,
                # early stop published by the controller kernels (no per-step queue marker / copy)
                publish=knobs.get_int("MACBF_PUBLISH", 1),
                poll_query_ms=100))
            if pw.ctrl_v.numel() < 352 or pw.ctrl_w.numel() < (c["f_node"] + 54) * 512 * (2 if pw.x3 else 1):
                raise native.NativeError("packed controller weights too small")
            if overlap and (self.hbuf.numel() < 2 * T * BNK or self.src.numel() < 2 * T * BNK):
                raise native.NativeError("CBF evaluation buffers too small")
            self._drv = native.lib().RolloutDriver(c)
        return self._drv

    def _rollout_steps(self, early_stop):
        """Rollout from the loaded inputs. early_stop=False: all Tmax steps, no host round trip
        (done envs are masked by the validity mask; used by the captured graph)."""
        cfg = self.tr.cfg
        B, N, K, D = self.B, self.N, self.K, self.D
        pw = self.pw
        if self._sums_dirty or self.graph_mode or torch.cuda.is_current_stream_capturing():
            self.cnt.zero_()
            self.safe.zero_()
            self.dist.zero_()
            self.act.zero_()
        self._sums_dirty = True
        events = []
        T = self.Tmax
        tail_scanned = False
        cur = torch.cuda.current_stream(self.dev)
        overlap = self.dedup and self.overlap_hfwd
        # the native drivers keep the node activations (node_acts); the Python loop does not
        self._acts_valid = bool(self.node_acts is not None and self.native_rollout and
                                not torch.cuda.is_current_stream_capturing())
        if self.native_rollout and not torch.cuda.is_current_stream_capturing():
            if self.small_rollout:
                # one persistent launch for the whole rollout (csrc/ctrl.hip rollout_small_kernel)
                # (step(): the registered backward graph of the horizon is launched by the driver
                # as soon as the horizon arrives -- _backward_graphed then skips its replay)
                # (sc None: load_inputs already wrote S[0] / G -- graph mode's warm-up)
                sc, self._scenario = self._scenario, None
                T, tail_scanned, launched = self._driver().run_small(
                    cur.cuda_stream, bool(early_stop), self._graph_launch,
                    native.ptr(sc[0]) if sc else 0, native.ptr(sc[1]) if sc else 0)
                self._launched_T = T if launched else None
                return self._tail_scan(T, tail_scanned)
            # the per-step launch loop in C++ (csrc/runtime.cpp): same launches, same order
            T, tail_scanned = self._driver().run(cur.cuda_stream, self.hstream.cuda_stream if overlap else 0,
                                                 self.copy_stream.cuda_stream, bool(early_stop))
            return self._tail_scan(T, tail_scanned)
        if overlap:
            self.hstream.wait_stream(cur)
        for t in range(self.Tmax):
            if overlap and t >= 1:
                # CBF h of step t-1's main slots on a side stream, concurrent with this step
                # (launched one step late: the slice of a step beyond the early stop is never issued)
                self._hfwd_slice(t - 1, cur)
            # the Hilbert order is refreshed every resort_every steps (agents move ~v*dt per
            # step: a slightly stale order only loosens the culling; results are identical)
            native.scan(self.S[t], self.idx[t], self.dang[t], self.cnt[t], self.safe[t], K=K,
                        do_knn=True, do_safety=cfg.compute_safety, n_agents=N,
                        prev_idx=self.idx[t - 1] if t > 0 else None, sort=t % self.resort_every == 0)
            native.ctrl_fwd(self.S[t], self.G, self.idx[t], pw.ctrl_w, pw.ctrl_off["ew1f"], pw.ctrl_off["nw1f"],
                            pw.ctrl_v, self.A[t], self.S[t + 1], self.dist[t], self.act[t], noise_t=t, **self._noise_args(),
                            pooled=self.pooled[t], argmax=self.argmax[t], prec=self.prec)
            if early_stop:
                # the per-env goal distances go to pinned host memory on a side stream (the
                # blit stays off the compute queue's critical path)
                done_ev = torch.cuda.Event()
                done_ev.record()
                self.copy_stream.wait_event(done_ev)
                with torch.cuda.stream(self.copy_stream):
                    self.host_dist[t].copy_(self.dist[t], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.copy_stream)
                events.append(ev)
                # 1-step-lagged host check: never stalls the queue on the step just issued
                if t >= 1:
                    events[t - 1].synchronize()
                    if self._all_done(t - 1):
                        # every env was done after step t-1: the trajectory is steps 0..t-1 (as
                        # in train.py:78-81). Step t was already issued; its scan already gave
                        # the kNN graph / safety of the final state s_t, its controller step is
                        # simply not used.
                        T = t
                        tail_scanned = True
                        break
        if overlap:
            if not tail_scanned:
                self._hfwd_slice(T - 1, cur)
            cur.wait_stream(self.hstream)
        return self._tail_scan(T, tail_scanned)

    def _tail_scan(self, T, tail_scanned):
        cfg = self.tr.cfg
        if (cfg.compute_safety or not self.reuse) and not tail_scanned:
            # safety of the final state; with reuse_nbr_idx=False also the kNN graph of s_T (for h')
            native.scan(self.S[T], self.idx[T] if not self.reuse else None, None, None,
                        self.safe[T] if cfg.compute_safety else None, K=self.K, do_knn=not self.reuse,
                        do_safety=cfg.compute_safety, n_agents=self.N,
                        prev_idx=self.idx[T - 1] if (not self.reuse and T > 0) else None)
        return T

    def _hfwd_slice(self, t, cur):
        """h / radius mask of the main slots of step t (evaluations [t*BNK, (t+1)*BNK) of the
        deduplicated list: they do not depend on the match) on the side stream."""
        ev = torch.cuda.Event()
        ev.record(cur)
        self.hstream.wait_event(ev)
        BNK = self.B * self.N * self.K
        pw = self.pw
        idx = self.idx[: t + 1]
        with torch.cuda.stream(self.hstream):
            native.cbf_hfwd(self.S, idx, idx, self.src, self.nev_host, pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_rm,
                            pw.cbf_v, self.hbuf, self.hmask, u_begin=t * BNK, u_end=(t + 1) * BNK, prec=self.prec)

    def _all_done(self, t):
        # the float arithmetic of rollout_stats_kernel / the native driver
        d = (self.host_dist[: t + 1].double() / native.FX_DIST).float() / float(self.N) < C.DIST_MIN_CHECK
        return bool(d.any(0).all())

    def trajectory(self, T: int) -> dict:
        """The last rollout of T steps in the oracle's layout (``oracle.rollout(forced=...)``):
        agent states (B, T+1, N, 2D), neighbour graphs (B, T, N, K) and the controller's
        max-pool argmax slots (B, T, N, 128) -- tests replay it through the oracle."""
        N = self.N
        S = native.from_records(self.S[: T + 1, :, :N]).transpose(0, 1).contiguous()
        return {"S": S, "idx": self.idx[:T].transpose(0, 1).long().contiguous(),
                "slots": self.argmax[:T].transpose(0, 1).contiguous()}

    # ------------------------------------------------------------------ step
    def step(self, s0, g, obs=None):
        if self.graph_mode:
            return self._step_graph(s0, g, obs)
        tm = self.tr.timer
        graphed = self._bwd_graph_on()
        if graphed:
            self.flush_stats()                      # a replay rewrites raw_stats
            self._graph_launch = self._graph_table == self._graph_suffix() and self._drv_launch
        try:
            # (a high-priority stream for this critical chain was measured slower: 7.62 -> 8.06 ms)
            T = self.rollout(s0, g, obs)
        finally:
            self._graph_launch = False
        tm.mark("rollout")
        if graphed:
            return self._backward_graphed(T)
        valid = self._counts(T)
        # the count all-reduce (the only mid-step collective) overlaps the parts of the backward
        # that do not read the global counts (reverse CSR, match, extra h evaluations)
        work = self.tr.dp.all_reduce_async(self.counts)
        tm.mark("counts")
        return self._stats(*self._backward(T, valid, counts_work=work))

    # ------------------------------------------------------------------ per-T backward graphs
    def _bwd_graph_on(self):
        return (self.bwd_graph and self.small_rollout and self.native_bptt and self.bptt and not self.graph_mode
                and not self.tr.dp.enabled and not self.tr.timer.enabled and not torch.cuda.is_current_stream_capturing())

    def _backward_graphed(self, T):
        """_counts + _backward for horizon T from a HIP graph captured the first time T occurs (that
        iteration runs eagerly, then the graph is captured: same kernels, same arguments -- every
        buffer is allocated once per engine, the statistics row is the fixed raw_stats, copied to a
        ring row after the replay)."""
        key = (int(T),) + self._graph_suffix()
        launched, self._launched_T = self._launched_T == T, None
        g = self._bwd_graphs.get(key)
        if g is None:
            valid = self._counts(T)
            out = self._stats(*self._backward(T, valid))
            self._capture_bwd(T, key)
            return out
        if not launched:
            self.flush_stats()                      # the replay rewrites raw_stats
            g.replay()
        self._sums_dirty = False                   # the captured rollout_stats zeroed the sums
        row = self._next_row()
        # raw_stats -> row: by the optimizer's commit launch when the trainer takes it
        # (take_stats_src), else before the row is read or raw_stats is rewritten (flush_stats)
        self._stats_pending = row
        st = self._stats(row, T)
        st.flush = self.flush_stats
        return st

    def take_stats_src(self, row):
        """The fixed buffer the pending statistics row is still to be copied from (the caller's
        launch copies it), or None."""
        if self._stats_pending is not None and self._stats_pending is row:
            self._stats_pending = None
            return self.raw_stats
        return None

    def flush_stats(self):
        if self._stats_pending is not None:
            self._stats_pending.copy_(self.raw_stats)
            self._stats_pending = None

    def _capture_bwd(self, T, key):
        cur = torch.cuda.current_stream(self.dev)
        side = torch.cuda.Stream(device=self.dev)
        side.wait_stream(cur)
        if self._bwd_pool is None:
            self._bwd_pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        dirty = self._sums_dirty
        self._bwd_capture = True
        try:
            with torch.cuda.graph(g, pool=self._bwd_pool, stream=side):
                valid = self._counts(T)
                self._backward(T, valid)
        finally:
            self._bwd_capture = False
            self._sums_dirty = dirty
        cur.wait_stream(side)
        self._bwd_graphs[key] = g
        if self.small_rollout and self.native_rollout:
            # the driver's table of this key suffix: launched right after the rollout (run_small)
            execs = [0] * (self.Tmax + 1)
            for k, gk in self._bwd_graphs.items():
                if k[1:] == key[1:]:
                    execs[k[0]] = int(gk.raw_cuda_graph_exec())
            self._driver().set_bwd_graphs(execs)
            self._graph_table = key[1:]

    def _graph_suffix(self):
        # (the flat gradient's address too: a checkpoint load that rebinds the flat buffers gets a
        # fresh graph; every other captured buffer lives as long as the engine)
        return (self._gscale()[0], self.tr.fp.grad.data_ptr(), self.tr.fp.flat.data_ptr())

    # ------------------------------------------------------------------ graph mode
    def _step_graph(self, s0, g, obs):
        self.load_inputs(s0, g, obs)
        gs = self._gscale()[0]
        if self._graphs is None or self._graph_gs != gs:     # (re)capture when a host scale changes
            self._capture()
            self._graph_gs = gs
        self._graphs[0].replay()
        self.tr.dp.all_reduce_(self.counts)
        self._graphs[1].replay()
        return self._stats(*self._graph_stats)

    def _capture(self):
        T = self.Tmax
        tm = self.tr.timer
        en, tm.enabled = tm.enabled, False
        try:
            cur = torch.cuda.current_stream(self.dev)
            side = torch.cuda.Stream(device=self.dev)
            side.wait_stream(cur)
            with torch.cuda.stream(side):            # warm-up: lazy buffers, code objects
                self._rollout_steps(False)
                v = self._counts(T)
                self._backward(T, v)
            cur.wait_stream(side)
            pool = torch.cuda.graph_pool_handle()
            ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(ga, pool=pool):
                self._rollout_steps(False)
                self._graph_valid = self._counts(T)
            with torch.cuda.graph(gb, pool=pool):
                self._graph_stats = self._backward(T, self._graph_valid)
            self._graphs = (ga, gb)
        finally:
            tm.enabled = en

    def _counts(self, T):
        """Validity mask (T, B) uint8 and the pooled counts [n_dang, n_safe, n_act] of this rank
        (+ the local stats in self.local), one kernel: step t of env b counts iff the env was
        not done before t."""
        valid = self.valid_buf[:T]
        reset = None if self.graph_mode else (self.dist, self.cnt, self.safe, self.act)
        if reset is not None and not torch.cuda.is_current_stream_capturing():
            # the early-stop copies of dist[t] into pinned host memory run on copy_stream: the reset
            # below must not overwrite a row such a copy is still reading
            torch.cuda.current_stream(self.dev).wait_stream(self.copy_stream)
        native.rollout_stats(self.dist[:T], self.cnt[:T], self.safe[: T + 1], self.act[:T], valid,
                             self.counts, self.local, N=self.N, reset=reset)
        if reset is not None:
            self._sums_dirty = False
        return valid

    def _backward(self, T, valid, counts_work=None):
        tr = self.tr
        B, N, K, W, Nn = self.B, self.N, self.K, self.W, self.Nn
        pw = self.pw
        tm = tr.timer
        # loss scale of the upstream gradients (fp16: dynamic, trainer-owned; bf16: 1). Every
        # backward quantity is linear in it; the flat gradient is unscaled after the slab reduce.
        gs, gsd = self._gscale()
        valid_u8 = valid
        E = T * B * N * K
        # ---- reverse CSR of the step graphs (needs only idx): on the aux stream, concurrent with
        #      the CBF kernel below
        G1 = 0 if self.reuse else 1
        rptr = self.rptr[: (T + G1) * B]
        redges = self.redges[: (T + G1) * B]
        self.aux.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(self.aux):
            native.rev_csr(self.idx[: T + G1].view((T + G1) * B, N, K), rptr, redges, n_nodes=Nn)
            csr_done = torch.cuda.Event()
            csr_done.record(self.aux)
        S = self.S[: T + 1]
        idx = self.idx[:T]
        nbb = native.cbf_bwd_grid(2 * E, self.dev, self.prec if (self.dedup and self.cbf16) else None)
        part_cbf = self._buf(self._part_cbf, nbb, native.CBF_PARTIAL)
        dE = self.dE[: 2 * E * W].view(2, T, B, N, K, W)
        idx1 = None if self.reuse else self.idx[1: T + 1]
        map1 = None
        if self.dedup:
            # ---- CBF on the deduplicated evaluation list: h'(s_{t+1}) of a slot is the next
            #      step's h of the same pair; only unmatched pairs get an extra evaluation
            map1 = self.map1[:T]
            src = self.src[: 2 * E]
            nev = native.cbf_match(self.idx[: T + G1], T, map1, src, self.mcnt, recomputed=not self.reuse,
                                   nev=self.nev_dev)
            hb, hm, dh = self.hbuf[: 2 * E], self.hmask[: 2 * E], self.dhbuf[: 2 * E]
            # the main slots [0, E) were evaluated during the rollout (overlap_hfwd): extras only
            native.cbf_hfwd(S, idx, idx if self.reuse else idx1, src, nev, pw.cbf_w, pw.cbf_off["w1f"],
                            pw.cbf_rm, pw.cbf_v, hb, hm, u_begin=E if self.overlap_hfwd else 0, prec=self.prec)
            self._counts_ready(counts_work)
            native.cbf_dh(hb, hm, map1, src, nev, self.dang[:T], valid_u8, self.counts, dh, self.loss_part,
                          grad_scale=gs, blk_active=self.blk_active, gscale=gsd)
            # backward over the evaluations with a nonzero upstream gradient only (exact: the
            # others contribute zeros); node_reduce reads dE where dh != 0
            if self.cbf16:
                rec = self.rec_list[: 2 * E]
                nact = native.cbf_active(dh, nev, self.blk_active, None, nact=self.nact_dev, rec=rec, src=src,
                                         idx=idx, idx1=idx if self.reuse else idx1)
                native.cbf_bwd(S, idx, dh.view(2, T, B, N, K), pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_rm, pw.cbf_v,
                               passes=2, dE=dE, partial=part_cbf, num_blocks=nbb, idx1=idx if self.reuse else idx1,
                               src=src, nev=nev, nact=nact, prec=self.prec, rec=rec, wrm16=pw.cbf_rm16,
                               w16=pw.cbf_w16)
            else:
                act = self.act_list[: 2 * E]
                nact = native.cbf_active(dh, nev, self.blk_active, act, nact=self.nact_dev)
                native.cbf_bwd(S, idx, dh.view(2, T, B, N, K), pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_rm, pw.cbf_v,
                               passes=2, dE=dE, partial=part_cbf, num_blocks=nbb, idx1=idx if self.reuse else idx1,
                               src=src, nev=nev, act=act, nact=nact, prec=self.prec)
            # (the loss partials are reduced with the weight-gradient slabs after the BPTT)
        else:
            # ---- CBF: h, h', hinge losses, upstream grads and the full backward in ONE kernel
            self._counts_ready(counts_work)
            native.cbf_bwd(S, idx, None, pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_rm, pw.cbf_v, passes=2, dE=dE,
                           partial=part_cbf, num_blocks=nbb, fused=True, dang=self.dang[:T], valid=valid_u8,
                           counts=self.counts, idx1=idx1, grad_scale=gs, prec=self.prec, gscale=gsd)
        cur = torch.cuda.current_stream(self.dev)
        cur.wait_event(csr_done)
        # no-BPTT: s_t is a detached input, only h'(s_{t+1}) gradients reach a_t
        red = dict(T=T, B=B, N=N, K=K, passes=2, pass_mask=0 if self.bptt else 2, shift1=G1, n_nodes=Nn,
                   map1=map1, gate=self.dhbuf[: 2 * E] if self.dedup else None)
        # BPTT consumes dS from the last step down: reduce the last reduce_late steps first, the
        # rest on the aux stream concurrently with the first BPTT steps (no LDS: it co-resides
        # with the latency-bound controller-backward kernels)
        ts = T + 1 - self.reduce_late if (self.bptt and self.reduce_late and T + 1 > 2 * self.reduce_late) else 0
        red_done = None
        if ts:
            native.node_reduce(dE, rptr, redges, self.dS, t_range=(ts, T + 1), **red)
            self.aux.wait_stream(cur)
            with torch.cuda.stream(self.aux):
                native.node_reduce(dE, rptr, redges, self.dS, t_range=(0, ts), **red)
                red_done = torch.cuda.Event()
                red_done.record(self.aux)
        else:
            native.node_reduce(dE, rptr, redges, self.dS, **red)
        tm.mark("cbf")
        # (not inside a captured graph: the collectives stay eager around the graphs)
        split = self.tr.dp.enabled and self.bptt and not self.graph_mode and not torch.cuda.is_current_stream_capturing()
        if split:
            # the CBF range now: reduced slab -> flat gradient -> async all-reduce during the BPTT
            native.reduce_rows(part_cbf, self.red_cbf)
            lo, hi = self.grad_ranges["cbf"]
            native.grad_assemble(self.red_all, self.g_ptr[lo: hi + 1], self.g_src, tr.fp.grad[lo:hi], scale=1.0 / gs,
                                 gscale=gsd)
            self._grad_work = self.tr.dp.all_reduce_async(tr.fp.grad[lo:hi])
        # ---- controller backward
        if self.bptt:
            # BPTT through the rollout: G_t = dL/ds_t, reverse time
            rptr3 = rptr[: T * B].view(T, B, Nn + 1)
            redges3 = redges[: T * B].view(T, B, N * K)
            Gp = self.bptt_groups
            slab_rows = self.slab_rows
            if Gp == 1 and red_done is None and self.native_bptt:
                # the reverse-time launch loop in C++ (csrc/runtime.cpp): same launches, same order
                self._bdriver().run(T, gs * ACT_COEF, cur.cuda_stream, use_acts=self._acts_valid)
            elif Gp == 1:
                self._bptt_chain(T, slice(0, B), valid_u8, gs, rptr3, redges3, self.part_node[: self.nb_node],
                                 self.part_edge[: self.nb_edge], self.nb_node, self.nb_edge, red_done, ts, cur)
            else:
                # envs never interact: Gp independent reverse-time chains, one per env group and
                # stream, interleave their latency-bound kernels on the CUs
                Bg = B // Gp
                nbn, nbe = self.grp_nb
                for g in range(Gp):
                    st = cur if g == 0 else self.gstreams[g - 1]
                    if g:
                        st.wait_stream(cur)
                    with torch.cuda.stream(st):
                        self._bptt_chain(T, slice(g * Bg, (g + 1) * Bg), valid_u8, gs, rptr3, redges3,
                                         self.part_node[g * nbn:(g + 1) * nbn], self.part_edge[g * nbe:(g + 1) * nbe],
                                         nbn, nbe, red_done, ts, st)
                for st in self.gstreams:
                    cur.wait_stream(st)
        else:
            # no BPTT: the steps are independent -> ONE node + ONE edge backward launch over all
            # T*B (step, env) pairs, with dL/da_t = dt * dL/dv_{t+1} from h'(s_{t+1}) + action loss
            TB = T * B
            nb_n, nb_e, Gr, dP = self._nobptt_bufs(TB)
            D = self.D
            Gr[:TB].view(T, B, N, D).copy_(self.G.unsqueeze(0).expand(T, B, N, D))
            pn = self._buf(self._part_cbf_nb, ("n", nb_n), native.CTRL_NODE_PARTIAL)
            pe = self._buf(self._part_cbf_nb, ("e", nb_e), native.CTRL_EDGE_PARTIAL)
            native.ctrl_node_bwd(self.pooled[:T].view(TB, N, self.prow), self.S[:T].view(TB, Nn, W), Gr[:TB],
                                 self.A[:T].view(TB, N, D), self.dS[1: T + 1].view(TB, N, W), valid_u8.view(TB),
                                 pw.ctrl_rm, pw.node_rm_off, pw.ctrl_v, gs * ACT_COEF, dP[:TB], None, pn, nb_n,
                                 act_cnt=self.counts[2:3], prec=self.prec, init=True, gscale=gsd,
                                 wrm16=self._node16(TB * N))
            native.ctrl_edge_bwd(self.S[:T].view(TB, Nn, W), self.idx[:T].view(TB, N, K), self.argmax[:T].view(TB, N, 128),
                                 dP[:TB], pw.ctrl_w, pw.ctrl_off["ew1f"], pw.ctrl_off["ew2tn"], None, pe, nb_e, prec=self.prec,
                                 init=True)
            self._nb_parts = (pn, pe)
        tm.mark("bptt")
        # ---- weight-gradient slabs (+ the loss partials) -> flat grad, one reduction launch
        if self.bptt:
            rn, re_ = slab_rows
            if self.step_rows:
                rn, re_ = T * rn, T * re_
            pnode, pedge = self.part_node[:rn], self.part_edge[:re_]
        else:
            pnode, pedge = self._nb_parts
        jobs = ([(part_cbf, self.red_cbf, False)] if not split else []) + [(pnode, self.red_node, False),
                                                                           (pedge, self.red_edge, False)]
        if self.dedup:
            jobs.append((self.loss_part, self.loss_red, False))
        native.reduce_multi(jobs)
        # ---- stats: one raw device row per iteration (no per-statistic kernels), derived lazily on
        #      read; written by the assembly launch, which (single process) also runs the finite check
        sums = self.loss_red[:10] if self.dedup else self.red_cbf[native.CBF_P_LOSS: native.CBF_P_LOSS + 10]
        row = self.raw_stats if (self.graph_mode or self._bwd_capture) else self._next_row()
        stats = (sums, self.counts, self.local, row)
        ok = None if split else self.check_ok
        if split:
            lo, hi = self.grad_ranges["controller"]
            native.grad_assemble(self.red_all, self.g_ptr[lo: hi + 1], self.g_src, tr.fp.grad[lo:hi], scale=1.0 / gs,
                                 gscale=gsd, stats=stats)
        else:
            native.grad_assemble(self.red_all, self.g_ptr, self.g_src, tr.fp.grad, scale=1.0 / gs, gscale=gsd, ok=ok,
                                 stats=stats)
        tm.mark("grad_reduce")
        Tv = T if not self.graph_mode else (valid != 0).any(1).sum()
        return row, Tv

    def _next_row(self):
        if self._ring_pos == self._ring.shape[0]:
            self._ring = torch.empty_like(self._ring)
            self._ring_pos = 0
        row = self._ring[self._ring_pos]
        self._ring_pos += 1
        return row

    def _gscale(self):
        """(host upstream-gradient scale, device loss scale or None): fp16 training keeps its
        dynamic loss scale on the device (no host round trip per step)."""
        d = getattr(self.tr, "gscale_dev", None)
        if d is not None:
            return 1.0, d
        return float(self.tr.grad_scale), None

    def reduce_grad(self):
        """DP all-reduce of this step's flat gradient (Trainer.reduce_grad): the CBF range was issued
        asynchronously before the BPTT (world > 1, BPTT); the rest is reduced here, then both are
        joined on the current stream."""
        dp = self.tr.dp
        work, self._grad_work = self._grad_work, None
        if work is None:
            dp.all_reduce_(self.tr.fp.grad)
            return
        lo, hi = self.grad_ranges["controller"]
        dp.all_reduce_(self.tr.fp.grad[lo:hi])
        work.wait()

    def _bdriver(self):
        """The native BPTT driver over this engine's persistent buffers (checked here once)."""
        if self._bdrv is None:
            B, N, Nn, K, D, W, T = self.B, self.N, self.Nn, self.K, self.D, self.W, self.Tmax
            G1 = 0 if self.reuse else 1
            exp = {"pooled": (self.pooled, self.hdt, (T, B, N, self.prow)), "S": (self.S, torch.float32, (T + 1, B, Nn, W)),
                   "G": (self.G, torch.float32, (B, N, D)), "A": (self.A, torch.float32, (T, B, N, D)),
                   "dS": (self.dS, torch.float32, (T + 1, B, N, W)), "Gb": (self.Gb, torch.float32, (T + 1, B, N, W)),
                   "valid": (self.valid_buf, torch.uint8, (T, B)), "idx": (self.idx, torch.int32, (T + G1, B, N, K)),
                   "argmax": (self.argmax, torch.uint8, (T, B, N, 128)),
                   "rptr": (self.rptr, torch.int32, ((T + G1) * B, Nn + 1)),
                   "redges": (self.redges, torch.int32, ((T + G1) * B, N * K)),
                   "act_scale": (self.counts[2:3], torch.float32, (1,)), "dP": (self.dP, self.hdt, (B, N, self.prow)),
                   "ego": (self.ego, torch.float32, (B, N, W)), "dEc": (self.dEc, torch.float32, (2, B, N, K, W))}
            for name, (t, dt, shape) in exp.items():
                native.check(t, dt, shape, name)
            rows = T if self.step_rows else 1
            if self.part_node.shape[0] < rows * self.nb_node or self.part_edge.shape[0] < rows * self.nb_edge:
                raise native.NativeError("controller slab buffers too small")
            pw = self.pw
            c = {k: native.ptr(v[0]) for k, v in exp.items()}
            c.update(dict(
                B=B, N=N, Nn=Nn, K=K, D=D, Tmax=T, prec=L.PREC_CODE[self.prec],
                nb_node=int(self.nb_node), nb_edge=int(self.nb_edge),
                qsplit=int(native.ctrl_edge_qsplit(B * N, self.dev)),
                part_node=native.ptr(self.part_node), part_edge=native.ptr(self.part_edge),
                ctrl_rm=native.ptr(pw.ctrl_rm), o_w1=int(pw.node_rm_off["w1"]), o_w2=int(pw.node_rm_off["w2"]),
                o_w3=int(pw.node_rm_off["w3"]), o_w4=int(pw.node_rm_off["w4"]), ctrl_v=native.ptr(pw.ctrl_v),
                ctrl_w=native.ptr(pw.ctrl_w), f_ew1f=int(pw.ctrl_off["ew1f"]), f_ew2tn=int(pw.ctrl_off["ew2tn"]),
                dt=float(C.TIME_STEP), sqrt3=float(C.SQRT3),
                node_chunk=int(native.node_bwd_chunk(B * N, self.dev)),
                step_rows=int(self.step_rows), node_part=native.CTRL_NODE_PARTIAL, edge_part=native.CTRL_EDGE_PARTIAL,
                node_acts=native.ptr(self.node_acts), node_act_bytes=native.node_act_bytes(self.prec),
                fused_step=int(native.bwd_step_fused(B * N, self.dev)),
                ctrl_w16=native.ptr(self.eb16_w) if self.eb16_w is not None else 0,
                node_rm16=native.ptr(self._node16(B * N)),
                gscale=native.ptr(getattr(self.tr, "gscale_dev", None))))
            self._bdrv = native.lib().BpttDriver(c)
        return self._bdrv

    def _bptt_chain(self, T, sl, valid_u8, gs, rptr3, redges3, part_node, part_edge, nbn, nbe, red_done, ts, st):
        """Reverse-time BPTT over the envs `sl` on stream `st`: G_t = dL/ds_t from G_{t+1}."""
        pw, K = self.pw, self.K
        step_rows = self.step_rows and sl == slice(0, self.B)
        for t in range(T - 1, -1, -1):
            pn, pe, init = part_node, part_edge, t == T - 1
            if step_rows:            # this step's own slab rows, written (not accumulated)
                r = T - 1 - t
                pn, pe, init = self.part_node[r * nbn:(r + 1) * nbn], self.part_edge[r * nbe:(r + 1) * nbe], True
            if red_done is not None and t == ts - 1:
                st.wait_event(red_done)                                # dS[0..ts) from the aux stream
            # G_{t+1}: the direct terms dS_T for t = T-1; else formed in the node kernel's prologue
            # from step t+1's records (fused BPTT combine, written to Gb[t+1])
            cmb = None
            if t < T - 1:
                cmb = dict(dS=self.dS[t + 1][sl], ego=self.ego[sl], dEc=self.dEc[(t + 1) & 1][sl], rptr=rptr3[t + 1][sl],
                           redges=redges3[t + 1][sl], Gn=self.dS[T][sl] if t + 1 == T - 1 else self.Gb[t + 2][sl],
                           Gout=self.Gb[t + 1][sl], K=K)
            node = dict(pooled=self.pooled[t][sl], S=self.S[t][sl], G=self.G[sl], A=self.A[t][sl], Gn=self.dS[T][sl],
                        valid_t=valid_u8[t][sl], wrm=pw.ctrl_rm, offs=pw.node_rm_off, wvec=pw.ctrl_v,
                        act_coef=gs * ACT_COEF, dP=self.dP[sl], ego=self.ego[sl], partial=pn,
                        act_cnt=self.counts[2:3], prec=self.prec, init=init,
                        gscale=getattr(self.tr, "gscale_dev", None), combine=cmb)
            edge = dict(S=self.S[t][sl], idx=self.idx[t][sl], argmax=self.argmax[t][sl], dP=self.dP[sl], wpack=pw.ctrl_w,
                        f_ew1f=pw.ctrl_off["ew1f"], f_ew2tn=pw.ctrl_off["ew2tn"], dEc=self.dEc[t & 1][sl], partial=pe,
                        prec=self.prec, init=init)
            if nbn == nbe and native.bwd_step_fused(self.G[sl].shape[0] * self.N, self.dev):
                native.ctrl_bwd_step(node, edge, nbn)            # node + edge backward: one launch
            else:
                native.ctrl_node_bwd(**node, num_blocks=nbn, wrm16=self._node16(self.G[sl].shape[0] * self.N))
                native.ctrl_edge_bwd(**edge, num_blocks=nbe, w16=self.eb16_w)

    def _node16(self, total_agents):
        """The 16x16x32 node-backward images if this engine runs that kernel (a launch over
        total_agents >= (B / groups) x N agents then takes 128-agent chunks too)."""
        if self.node16_w is not None and native.node_bwd_chunk(total_agents, self.dev) != 128:
            raise native.NativeError("16x16x32 node backward: a launch without 128-agent chunks")
        return self.node16_w

    def _counts_ready(self, work):
        """Join the (async) count all-reduce (the node backward reads the action-loss count
        counts[2] on the device: no host sync)."""
        if work is not None:
            work.wait()

    def _stats(self, raw, T):
        from ..utils.metrics import StepStats
        if self.graph_mode:      # the captured graph writes fixed buffers
            return StepStats(raw.clone(), T.clone() if isinstance(T, torch.Tensor) else T)
        return StepStats(raw, T)

    def _buf(self, cache, key, cols):
        b = cache.get(key)
        if b is None:
            rows = key[1] if isinstance(key, tuple) else key
            b = torch.zeros(rows, cols, dtype=torch.float32, device=self.dev)
            cache[key] = b
        return b

    def _nobptt_bufs(self, TB):
        """(T*B)-batched buffers for the no-BPTT controller backward (sized for Tmax)."""
        if "dP" not in self._nobptt:
            TBm = self.Tmax * self.B
            nb_n, nb_e = native.ctrl_bwd_grids(TBm * self.N, self.dev, self.prec, eb16=self.eb16_w is not None)
            self._nobptt = {
                "grids": (nb_n, nb_e),
                "G": torch.zeros(TBm, self.N, self.D, dtype=torch.float32, device=self.dev),
                "dP": torch.zeros(TBm, self.N, self.prow, dtype=self.hdt, device=self.dev),
            }
        nb_n, nb_e = self._nobptt["grids"]
        return nb_n, nb_e, self._nobptt["G"], self._nobptt["dP"]
