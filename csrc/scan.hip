// K1: per-step all-pairs scan of one timestep graph (B envs x N agents), gfx950.
//
// One pass over all candidate agents j of the env (positions+velocities staged in LDS in
// 1024-agent tiles, read as wave-wide broadcasts) produces, per agent i:
//   * the top-K nearest neighbours (self at slot 0, ties -> lower index), kept sorted in
//     registers with a statically unrolled insertion (reference core.py:234-250, which
//     builds a dense (N,N,C) tensor and topk's it 3x per step -- never materialised here);
//   * the training TTC danger bit of each kept edge (core.py:187-209: r=DIST_MIN_THRES,
//     ttc=TIME_TO_COLLISION) and per-env dangerous/safe edge counts (loss normalisers);
//   * the all-pairs safety flag (core.py:212-231 / train.py:74-75: r=DIST_MIN_CHECK,
//     ttc=TIME_TO_COLLISION_CHECK) -> per-env count of safe agents.
// fp contraction is OFF in this file so distances / TTC decisions are bit-identical to the
// PyTorch oracle (separately rounded products, same association order).
#pragma clang fp contract(off)
#include <cstdlib>
#include "common.h"
#include "args.h"
#include "state.h"
#include "ttc.h"

namespace mb {


// ---------------------------------------------------------------------------------------
// Spatial ordering. The top-K insertion is wave-divergent: a wave pays for the 12-step
// insertion whenever ANY of its 64 lanes inserts. With agents in random order every
// candidate is an insertion for some lane. cell_sort_kernel orders each env's agents along a
// Hilbert curve (32x32 grid over the scenario square), so a wave's 64 agents are spatial
// neighbours; scan_kernel then visits candidates outward from the wave's own position on
// the curve, the lists converge within the first ~100 candidates and later candidates
// almost never insert. Results do not depend on the order: (d2, index) is compared
// lexicographically, so idx/dang/counts/safety are exactly those of the plain all-pairs scan.
// ---------------------------------------------------------------------------------------
constexpr int SORT_BLOCK = 1024;
constexpr int CURVE_BINS = 1024;

// Hilbert index on the 32x32 cell grid: consecutive indices are edge-adjacent cells, so any
// 64 consecutive agents cover a compact patch (a Morton range can jump across the square).
DEV int hilbert32(int x, int y) {
  int d = 0;
#pragma unroll
  for (int s = 16; s > 0; s >>= 1) {
    const int rx = (x & s) ? 1 : 0;
    const int ry = (y & s) ? 1 : 0;
    d += s * s * ((3 * rx) ^ ry);
    if (ry == 0) {
      if (rx == 1) { x = 31 - x; y = 31 - y; }
      const int t = x; x = y; y = t;
    }
  }
  return d;
}

// cell coordinate 0..31 of a scaled position; NaN (a diverged state) and out-of-range values clamp
// (a float -> int conversion of NaN / out-of-range values is undefined)
DEV int grid_cell(float x) { return x >= 1.f ? (x < 31.f ? (int)x : 31) : 0; }

__global__ __launch_bounds__(SORT_BLOCK) void cell_sort_kernel(CellSortArgs a) {
  __shared__ int hist[CURVE_BINS];
  __shared__ int wsum[SORT_BLOCK / WAVE];
  const int b = blockIdx.x;
  const int R = a.rec;                                  // float4s per node record
  const float4* Sb = a.S + (long)b * a.s_env * R;
  for (int q = threadIdx.x; q < CURVE_BINS; q += SORT_BLOCK) hist[q] = 0;
  __syncthreads();
  const float inv = 32.f / a.L;
  for (int i = threadIdx.x; i < a.N; i += SORT_BLOCK) {
    const float4 s = Sb[i * R];
    const int cx = grid_cell(s.x * inv);
    const int cy = grid_cell(s.y * inv);
    atomicAdd(&hist[hilbert32(cx, cy)], 1);
  }
  __syncthreads();
  // exclusive scan of 1024 bins with 1024 threads: wave scan + wave totals
  const int lane = threadIdx.x & 63, w = threadIdx.x / WAVE;
  int v = hist[threadIdx.x];
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int q = 0; q < SORT_BLOCK / WAVE; ++q) { const int t = wsum[q]; wsum[q] = acc; acc += t; }
  }
  __syncthreads();
  hist[threadIdx.x] = x - v + wsum[w];
  __syncthreads();
  int* perm = a.perm + (long)b * a.N;
  for (int i = threadIdx.x; i < a.N; i += SORT_BLOCK) {
    const float4 s = Sb[i * R];
    const int cx = grid_cell(s.x * inv);
    const int cy = grid_cell(s.y * inv);
    const int p = atomicAdd(&hist[hilbert32(cx, cy)], 1);
    perm[p] = i;
  }
}

// Block = BS/64 waves x 64/LPA agents (consecutive on the curve), LPA lanes each. BS = 256 for
// envs up to 512 nodes; SCAN_BS_BIG above (the whole env is staged per block: bigger blocks
// amortise it; a 4096-node env stages 128 KiB, one 16-wave block per CU).
constexpr int SCAN_MAXN = 4096;      // whole env staged in LDS
constexpr int SCH = 8;               // candidates per chunk (one bounding box each)
constexpr int SSC = 8;               // chunks per superchunk (second culling level)

static inline size_t scan_lds_bytes(int Nn) {
  const int Np = (Nn + SCH - 1) / SCH * SCH;
  const int nch = Np / SCH, nsc = (nch + SSC - 1) / SSC;
  return (size_t)Np * 32 + (size_t)nch * 32 + (size_t)nsc * 32 + (size_t)Np * 2;   // + pinv (u16)
}

constexpr uint64_t KEY_EMPTY = (0x7f800000ull << 32) | 0xffffffffull;   // (+inf, max index)

template <int K>
DEV void topk_insert(uint64_t (&bk)[K], uint64_t x) {
  // caller guarantees x < bk[K-1]; bk is sorted ascending, so c[] is monotone
  bool c[K];
#pragma unroll
  for (int q = 0; q < K; ++q) c[q] = x < bk[q];
#pragma unroll
  for (int q = K - 1; q >= 1; --q) bk[q] = c[q - 1] ? bk[q - 1] : (c[q] ? x : bk[q]);
  bk[0] = c[0] ? x : bk[0];
}

// Merge of two ascending key lists of length K into the K smallest keys of both, ascending, by
// a bitonic network (lists padded to P = 2^ceil(log2 K) with KEY_EMPTY): c[i] = min(a[i],
// b[P-1-i]) holds the P smallest keys of the union as a bitonic sequence, log2 P half-cleaner
// stages sort it. Branch-free and fixed cost (P mins + P/2 log2 P compare-exchanges), where the
// insertion merge ran up to K wave-divergent K-step insertions per butterfly level. Keys are
// unique, so the result equals the insertion merge's.
template <int K>
DEV void topk_merge(uint64_t (&bk)[K], const uint64_t (&px)[K]) {
  constexpr int P = K <= 1 ? 1 : K <= 2 ? 2 : K <= 4 ? 4 : K <= 8 ? 8 : 16;
  uint64_t c[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const uint64_t x = i < K ? bk[i] : KEY_EMPTY;
    const uint64_t y = (P - 1 - i) < K ? px[P - 1 - i] : KEY_EMPTY;
    c[i] = x < y ? x : y;
  }
#pragma unroll
  for (int st = P / 2; st >= 1; st >>= 1) {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      if ((i & st) == 0) {
        const uint64_t x = c[i], y = c[i + st];
        const bool sw = y < x;
        c[i] = sw ? y : x;
        c[i + st] = sw ? x : y;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < K; ++i) bk[i] = c[i];
}

DEV float wave_min(float v) { return -wave_max(-v); }

// Chunked scan with conservative culling. The env's graph nodes (agents, then static
// obstacle points) are staged in curve order in LDS with a bounding box (+ max speed) per
// chunk of 8. A wave compares the box gap to its own box (over its agent lanes): the whole
// chunk is skipped for kNN when the gap exceeds every lane's current K-th distance (strictly,
// so ties are never skipped), and for the safety check when it exceeds the reachable distance
// r + ttc*(vmax_wave + vmax_chunk) (x1.01 + 1e-4 margin). Both decisions are wave-uniform
// branches; after the local neighbourhood has filled the lists almost every far chunk costs
// one box test instead of 8 pair evaluations. Obstacle nodes are candidates, never centres.
// xor-shuffle of a lane value across the LPA lanes of one agent (o = 32: v_permlane32_swap)
DEV float grp_xor(float v, int o) { return __uint_as_float(lane_xor_rt(__float_as_uint(v), o)); }
DEV unsigned grp_xoru(unsigned v, int o) { return lane_xor_rt(v, o); }

// Large envs (Nn > SCAN_MAXN, the whole env no longer fits LDS): scan_stage_kernel writes the
// curve-ordered node arrays and the chunk / superchunk boxes of every env ONCE per step to a
// global workspace [tp Np | tv Np | cbl nch | cbh nch | sbl nsc | sbh nsc]; scan_kernel<GLB>
// copies only the boxes to LDS (the culling runs from LDS) and reads the candidate nodes of the
// surviving chunks from global memory (L2-resident; wave-uniform addresses). Same results.
constexpr int STAGE_BLOCK = 256;                 // chunks per stage block (a multiple of SSC)

template <int D>
__global__ __launch_bounds__(STAGE_BLOCK) void scan_stage_kernel(ScanArgs a) {
  __shared__ float4 lbl[STAGE_BLOCK], lbh[STAGE_BLOCK];
  const int Nn = a.Nn;
  const int Np = (Nn + SCH - 1) / SCH * SCH;
  const int nch = Np / SCH, nsc = (nch + SSC - 1) / SSC;
  const int b = blockIdx.y;
  float4* w = a.ws + (long)b * a.ws_env;
  float4 *tp = w, *tv = w + Np, *cbl = tv + Np, *cbh = cbl + nch, *sbl = cbh + nch, *sbh = sbl + nsc;
  const float4* Sb = a.S + (long)b * a.s_env * REC<D>;
  const int* perm = a.perm + (long)b * Nn;
  const int c = blockIdx.x * STAGE_BLOCK + threadIdx.x;
  float4 lo = make_float4(INFINITY, INFINITY, INFINITY, 0.f);
  float4 hi = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
  if (c < nch) {
#pragma unroll
    for (int u = 0; u < SCH; ++u) {
      const int q = c * SCH + u;
      if (q < Nn) {
        const int id = perm[q];
        float p[D], v[D];
        load_rec<D>(Sb, (unsigned)id, p, v);
        const float z = (D == 3) ? p[D - 1] : 0.f;
        const float vz = (D == 3) ? v[D - 1] : 0.f;
        const float4 s = make_float4(p[0], p[1], z, __int_as_float(id));
        const float vm = sqrtf(sqsum<D>(v));
        tp[q] = s;
        tv[q] = make_float4(v[0], v[1], vz, vm);
        lo.x = fminf(lo.x, s.x); lo.y = fminf(lo.y, s.y); lo.z = fminf(lo.z, s.z);
        hi.x = fmaxf(hi.x, s.x); hi.y = fmaxf(hi.y, s.y); hi.z = fmaxf(hi.z, s.z);
        lo.w = fmaxf(lo.w, vm);
      } else {
        tp[q] = make_float4(INFINITY, INFINITY, INFINITY, __int_as_float(-1));
        tv[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    cbl[c] = lo;
    cbh[c] = hi;
  }
  lbl[threadIdx.x] = lo;
  lbh[threadIdx.x] = hi;
  __syncthreads();
  const int sc = blockIdx.x * (STAGE_BLOCK / SSC) + threadIdx.x;
  if (threadIdx.x < STAGE_BLOCK / SSC && sc < nsc) {
    float4 sl = make_float4(INFINITY, INFINITY, INFINITY, 0.f);
    float4 sh = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
    for (int u = threadIdx.x * SSC; u < threadIdx.x * SSC + SSC && blockIdx.x * STAGE_BLOCK + u < nch; ++u) {
      const float4 l = lbl[u], q = lbh[u];
      sl.x = fminf(sl.x, l.x); sl.y = fminf(sl.y, l.y); sl.z = fminf(sl.z, l.z); sl.w = fmaxf(sl.w, l.w);
      sh.x = fmaxf(sh.x, q.x); sh.y = fmaxf(sh.y, q.y); sh.z = fmaxf(sh.z, q.z);
    }
    sbl[sc] = sl;
    sbh[sc] = sh;
  }
}

// SCAN_WAVE_ATOMIC (A/B build knob): the per-env counts added by every wave instead of one
// block-level sum after a barrier
constexpr int SCAN_WAVE_ATOMIC = 0;
// 3-D scenes: on (round 5: the 3-D candidate loop varies 1.8x between waves of a block, and with
// the barrier a wave waited for the block's slowest; with SCAN_BS_BIG3 = 512 config #5 fp16
// 9.26-9.28 -> 8.54-8.56 ms, fp32 13.70 -> 13.05, interleaved, profiles/r5_b15/); 2-D: off
// (+0.04 ms at the headline, profiles/r5_b14/)
constexpr int SCAN_WAVE_ATOMIC3 = 1;

// SCAN_CELL3 / SCAN_CELL2 (A/B build knobs): with a temporal bound, search a uniform cell grid of
// the env around each agent instead of the wave-uniform chunk culling. The 2-D curve order leaves
// every 3-D chunk a full-height column and every 3-D wave box as tall as the env, so a 3-D wave
// evaluates ~2x the chunks of a 2-D one (stamps_scan.py: 30 vs 14); and in either dimension a wave
// evaluates a chunk when ANY of its 16 agents needs it. With cells, each agent's four lanes visit
// only the cell rows within its own bound (the largest current distance of its previous K
// neighbours) and safety reach. Same keys, same exact tests: the same lists, bits and counts.
// 3-D: on (round 5: config #5 scan 93.6 -> 72.0 us per call, fp16 8.57 -> 8.12 ms over the cell
// versions, interleaved, profiles/r5_b27/ - r5_b32/)
constexpr int SCAN_CELL3 = 1;
// 2-D: on (round 5: scan 47.1 -> 33.8 us per call, candidate loop 50 -> 25 k cycles per wave,
// headline fp32 10.52-10.53 -> 10.26-10.27 ms, bf16 6.65 -> 6.39, interleaved, profiles/r5_b25/)
constexpr int SCAN_CELL2 = 1;
// 3-D: 10^3 cells (~1.1 graph nodes per cell at config #5; two cells per thread in the prefix sum
// of the 512-thread blocks). Config #5 fp16, interleaved: 8^3 8.144 / 8.093, 10^3 8.083 / 8.101,
// 12^3 8.565 / 8.575 ms (its LDS leaves one block per CU); candidates per wave 674 -> 552
// (profiles/r5_b35/)
constexpr int SCAN_CELL_G3 = 10;
// 2-D: 24^2 cells (~1.8 agents per cell at the headline) in blocks of >= 576 threads (one thread
// per cell in the prefix sum), 16^2 in smaller blocks. Round 5, with the row-table walk, headline
// fp32 interleaved: 16^2 10.205 / 10.190, 24^2 10.173 / 10.150, 32^2 10.184 / 10.152 ms
// (candidates per wave 479 / 372 / 323, profiles/r5_b33/); on a second box 10.118 / 10.152 vs
// 10.122 / 10.112, bf16 6.255 vs 6.238, slice unchanged (profiles/r5_b34/)
constexpr int SCAN_CELL_G2 = 24;
template <int D, int BS> constexpr int cell_g() {
  return D == 3 ? SCAN_CELL_G3 : (BS >= SCAN_CELL_G2 * SCAN_CELL_G2 ? SCAN_CELL_G2 : 16);
}
template <int D, int BS> constexpr int cell_n() {
  return D == 3 ? cell_g<3, BS>() * cell_g<3, BS>() * cell_g<3, BS>() : cell_g<2, BS>() * cell_g<2, BS>();
}
template <int D> constexpr bool cell_on() { return D == 3 ? SCAN_CELL3 != 0 : SCAN_CELL2 != 0; }
// cell arrays: [NCELL + 1] starts | [NCELL] fill counters | [Np] curve positions (u16) | [Np]
// node records (x, y, z, id) in cell order (16-byte aligned: one LDS read per candidate)
// SCAN_CELL_VZ: cell records carry the node's speed (2-D: in the unused z slot; 3-D: rounded up to
// bf16 beside a 16-bit node id), so the safety pre-test of a candidate needs no second (dependent)
// LDS read
constexpr int SCAN_CELL_VZ = 1;
// rows of an agent's search box per row-table batch (more rows: further batches)
constexpr int SCAN_RT = 16;
template <int D, int BS> static inline size_t scan_cell_lds(int Np, int nag) {
  return ((size_t)(2 * cell_n<D, BS>() + 1) * 4 + (size_t)Np * 2 + 15) / 16 * 16 + (size_t)Np * 16 + 16 +
         (size_t)nag * SCAN_RT * 4;
}
// cell coordinate of a scaled position (monotone; NaN and values below 0 -> 0, above -> G-1)
template <int G> DEV int cell_coord(float x) { return x >= 1.f ? (x < (float)(G - 1) ? (int)x : G - 1) : 0; }

// SCAN_THR_SKIP: the per-chunk threshold update (group min + wave max) only when some lane of the
// wave inserted into its list in that chunk, the all-danger update only when some lane's danger
// flag turned on; the same lists, bits and counts either way (default since round 5: scan 48.8 ->
// 47.5 us, headline -0.04 ms, config #5 fp16 9.42-9.43 -> 9.30-9.33 ms, profiles/r5_b12/)

// GLB: 0 = env staged in LDS; 1 = nodes in the global workspace, culling boxes copied to LDS;
// 2 = boxes read from the workspace too (envs whose boxes exceed LDS: > ~36 K nodes)
constexpr int SCAN_STAGE_BT = 4;
// ST (diagnostics): per-wave phase clocks and chunk counts to a.stamps[(block * BS/64 + wave) * 16 + k]:
// 0 env staging, 1 culling boxes, 2 wave setup + temporal bound, 3 candidate loop, 4 list merge,
// 5 output slots, 6 counts; 8 superchunks visited, 9 chunks tested, 10 chunks evaluated,
// 11 chunks with an insertion, 12 evaluated for the kNN, 13 for the safety test only
// (scripts/stamps_scan.py). A separate instantiation.
template <int K, int D, int BS, int LPA, int GLB, bool ST = false>
__global__ __launch_bounds__(BS) void scan_kernel(ScanArgs a) {
  unsigned long long ph[16] = {}, tck = ST ? __builtin_amdgcn_s_memtime() : 0ull;
  auto stamp = [&](int k) {
    if constexpr (ST) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      ph[k] += t - tck;
      tck = t;
    }
  };
  constexpr int APW = WAVE / LPA;                              // agents per wave
  constexpr int SCAN_AG = BS / LPA;                            // agents (curve positions) per block
  extern __shared__ float4 smem4[];
  const int N = a.N, Nn = a.Nn;
  const int Np = (Nn + SCH - 1) / SCH * SCH;
  const int nch = Np / SCH, nsc = (nch + SSC - 1) / SSC;
  __shared__ float red[3][BS / WAVE];
  // ROLL_XCD: the blocks of one env (consecutive in x) on one XCD (they stage the same env)
  const int lin0 = (int)(blockIdx.y * gridDim.x + blockIdx.x);
  const int lin = ROLL_XCD ? xcd_block(lin0, (int)(gridDim.x * gridDim.y)) : lin0;
  const int bx = lin % (int)gridDim.x;
  const int b = lin / (int)gridDim.x;
  float4 *tp, *tv, *cbl, *cbh, *sbl, *sbh;
  if constexpr (GLB) {
    tp = a.ws + (long)b * a.ws_env;                            // [Np] x, y, z, node id (global)
    tv = tp + Np;                                              // [Np] vx, vy, vz, |v| (global)
    cbl = GLB == 2 ? tv + Np : smem4;                          // boxes: LDS copies (GLB 1)
    cbh = cbl + nch;
    sbl = cbh + nch;
    sbh = sbl + nsc;
  } else {
    tp = smem4;                                                // [Np] x, y, z, node id (bits)
    tv = tp + Np;                                              // [Np] vx, vy, vz, |v|
    cbl = tv + Np;                                             // [nch] min x, y, z, max |v|
    cbh = cbl + nch;                                           // [nch] max x, y, z
    sbl = cbh + nch;                                           // [nsc] superchunk boxes
    sbh = sbl + nsc;
  }
  // LDS path: curve position of every node id, so the neighbour records the kernel needs after
  // the staging (the temporal bound's previous neighbours, the output slots' TTC test) come from
  // the staged LDS arrays instead of dependent global gathers
  unsigned short* pinv = reinterpret_cast<unsigned short*>(sbh + nsc);
  const float4* Sb = a.S + (long)b * a.s_env * REC<D>;
  const int* perm = a.perm + (long)b * Nn;
  constexpr int CG = cell_g<D, BS>(), NCELL = cell_n<D, BS>();
  constexpr bool CELLS = cell_on<D>() && !GLB;
  constexpr int MQ = (4096 + BS - 1) / BS;                     // cell path: staged nodes per thread
  const bool use_cells = CELLS && a.cells && a.prev_idx && a.do_knn && Nn <= MQ * BS;   // uniform per launch
  __shared__ float cgrid[8];                                   // lo.xyz, cells per unit.xyz, max |v|
  __shared__ float wbox[BS / WAVE][8];                         // per-wave bounding boxes (cell path)
  // this thread's running bounding box of its staged nodes (cell path: replaces the chunk boxes)
  float bx0 = INFINITY, by0 = INFINITY, bz0 = INFINITY, bx1 = -INFINITY, by1 = -INFINITY, bz1 = -INFINITY, bvm = 0.f;
  if constexpr (GLB == 2) {
  } else if constexpr (GLB == 1) {
    const float4* gb = tv + Np;
    for (int q = threadIdx.x; q < 2 * (nch + nsc); q += BS) cbl[q] = gb[q];
  } else
  // batches of SCAN_STAGE_BT positions per thread: the perm -> record chains of a batch are in
  // flight together (clamped indices, unconditional loads), not one dependent pair per iteration
  for (int q0 = threadIdx.x; q0 < Np; q0 += SCAN_STAGE_BT * BS) {
    int ids[SCAN_STAGE_BT];
#pragma unroll
    for (int u = 0; u < SCAN_STAGE_BT; ++u) ids[u] = perm[min(q0 + u * BS, Nn - 1)];
    float p[SCAN_STAGE_BT][D], v[SCAN_STAGE_BT][D];
#pragma unroll
    for (int u = 0; u < SCAN_STAGE_BT; ++u) load_rec<D>(Sb, (unsigned)ids[u], p[u], v[u]);
#pragma unroll
    for (int u = 0; u < SCAN_STAGE_BT; ++u) {
      const int q = q0 + u * BS;
      if (q >= Np) break;
      if (q < Nn) {
        const float z = (D == 3) ? p[u][D - 1] : 0.f;
        const float vz = (D == 3) ? v[u][D - 1] : 0.f;
        const float vm = sqrtf(sqsum<D>(v[u]));
        tp[q] = make_float4(p[u][0], p[u][1], z, __int_as_float(ids[u]));
        tv[q] = make_float4(v[u][0], v[u][1], vz, vm);
        pinv[ids[u]] = (unsigned short)q;
        if constexpr (CELLS) {
          bx0 = fminf(bx0, p[u][0]); by0 = fminf(by0, p[u][1]); bz0 = fminf(bz0, z);
          bx1 = fmaxf(bx1, p[u][0]); by1 = fmaxf(by1, p[u][1]); bz1 = fmaxf(bz1, z);
          bvm = fmaxf(bvm, vm);
        }
      } else {
        tp[q] = make_float4(INFINITY, INFINITY, INFINITY, __int_as_float(-1));   // key == KEY_EMPTY
        tv[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
  if constexpr (CELLS) {
    if (use_cells) {                          // every wave: its box to wbox (all lanes take part)
      bx0 = wave_min(bx0); by0 = wave_min(by0); bz0 = wave_min(bz0);
      bx1 = wave_max(bx1); by1 = wave_max(by1); bz1 = wave_max(bz1); bvm = wave_max(bvm);
      if ((threadIdx.x & (WAVE - 1)) == 0) {
        float* w = wbox[threadIdx.x / WAVE];
        w[0] = bx0; w[1] = by0; w[2] = bz0; w[3] = bx1; w[4] = by1; w[5] = bz1; w[6] = bvm;
      }
    }
  }
  __syncthreads();
  stamp(0);
  if constexpr (!GLB) {
  if (!use_cells) {                           // the chunk culling's boxes (the cell path needs none)
  for (int c = threadIdx.x; c < nch; c += BS) {
    float4 lo = make_float4(INFINITY, INFINITY, INFINITY, 0.f);
    float4 hi = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
#pragma unroll
    for (int u = 0; u < SCH; ++u) {
      const int q = c * SCH + u;
      if (q < Nn) {
        const float4 s = tp[q];
        lo.x = fminf(lo.x, s.x); lo.y = fminf(lo.y, s.y); lo.z = fminf(lo.z, s.z);
        hi.x = fmaxf(hi.x, s.x); hi.y = fmaxf(hi.y, s.y); hi.z = fmaxf(hi.z, s.z);
        lo.w = fmaxf(lo.w, tv[q].w);
      }
    }
    cbl[c] = lo;
    cbh[c] = hi;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < nsc; c += BS) {
    float4 lo = make_float4(INFINITY, INFINITY, INFINITY, 0.f);
    float4 hi = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
    for (int u = c * SSC; u < min(c * SSC + SSC, nch); ++u) {
      const float4 l = cbl[u], q = cbh[u];
      lo.x = fminf(lo.x, l.x); lo.y = fminf(lo.y, l.y); lo.z = fminf(lo.z, l.z); lo.w = fmaxf(lo.w, l.w);
      hi.x = fmaxf(hi.x, q.x); hi.y = fmaxf(hi.y, q.y); hi.z = fmaxf(hi.z, q.z);
    }
    sbl[c] = lo;
    sbh[c] = hi;
  }
  __syncthreads();
  }
  }
  // cell grid over the env's bounding box (SCAN_CELL2 / SCAN_CELL3): counting sort of the staged
  // curve positions by cell; the order inside a cell is irrelevant (the lists are exact for any order)
  int* cstart = reinterpret_cast<int*>(pinv + Np);             // [NCELL + 1] cell starts
  int* cfill = cstart + NCELL + 1;                             // [NCELL] fill counters
  unsigned short* clist = reinterpret_cast<unsigned short*>(cfill + NCELL);   // [Np] curve positions
  float4* ctp = reinterpret_cast<float4*>((reinterpret_cast<uintptr_t>(clist + Np) + 15) & ~(uintptr_t)15);   // [Np]
  unsigned* rtab = reinterpret_cast<unsigned*>(ctp + Np);      // [SCAN_AG][SCAN_RT] row ranges (s | e << 16)
  auto cell_of = [&](const float4& t) {
    const int cx = cell_coord<CG>((t.x - cgrid[0]) * cgrid[3]), cy = cell_coord<CG>((t.y - cgrid[1]) * cgrid[4]);
    if constexpr (D == 3) return (cell_coord<CG>((t.z - cgrid[2]) * cgrid[5]) * CG + cy) * CG + cx;
    return cy * CG + cx;
  };
  if constexpr (CELLS) {
    if (use_cells) {
      if (threadIdx.x < WAVE) {               // wave 0: bounding box and max speed of the env's nodes
        const int l = threadIdx.x;
        float4 lo = make_float4(INFINITY, INFINITY, INFINITY, 0.f), hi = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
        if (l < BS / WAVE) {
          const float* w = wbox[l];
          lo = make_float4(w[0], w[1], w[2], w[6]);
          hi = make_float4(w[3], w[4], w[5], 0.f);
        }
        lo.x = wave_min(lo.x); lo.y = wave_min(lo.y); lo.z = wave_min(lo.z); lo.w = wave_max(lo.w);
        hi.x = wave_max(hi.x); hi.y = wave_max(hi.y); hi.z = wave_max(hi.z);
        if (l == 0) {
          const float g = (float)CG;
          cgrid[0] = lo.x; cgrid[1] = lo.y; cgrid[2] = lo.z;
          cgrid[3] = g / fmaxf(hi.x - lo.x, 1e-6f); cgrid[4] = g / fmaxf(hi.y - lo.y, 1e-6f);
          cgrid[5] = g / fmaxf(hi.z - lo.z, 1e-6f);
          cgrid[6] = lo.w;
        }
      }
      for (int c = threadIdx.x; c < NCELL; c += BS) cfill[c] = 0;
      __syncthreads();
      // each node's cell and rank inside it (the atomic's return), kept for the scatter
      int crk[MQ];
#pragma unroll
      for (int u = 0; u < MQ; ++u) {
        const int q = threadIdx.x + u * BS;
        if (q < Nn) {
          const int c = cell_of(tp[q]);
          crk[u] = (c << 16) | atomicAdd(&cfill[c], 1);
        }
      }
      __syncthreads();
      // exclusive scan of the cell counts: PC consecutive cells per thread, wave scans of the
      // thread sums, then the wave totals
      constexpr int PC = (NCELL + BS - 1) / BS;
      __shared__ int wtot[BS / WAVE];
      const int tid = threadIdx.x, ln = tid & 63, wv = tid / WAVE;
      int loc[PC];
      int v = 0;
#pragma unroll
      for (int p = 0; p < PC; ++p) {
        const int c = tid * PC + p;
        loc[p] = v;
        v += c < NCELL ? cfill[c] : 0;
      }
      int x = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (ln >= o) x += y;
      }
      if (ln == 63) wtot[wv] = x;
      __syncthreads();
      {
        int pre = 0;
        for (int w = 0; w < wv; ++w) pre += wtot[w];
#pragma unroll
        for (int p = 0; p < PC; ++p) {
          const int c = tid * PC + p;
          if (c < NCELL) cstart[c] = pre + x - v + loc[p];
        }
        if (tid == BS - 1) cstart[NCELL] = pre + x;
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < MQ; ++u) {
        const int q = threadIdx.x + u * BS;
        if (q < Nn) {
          const int dst = cstart[crk[u] >> 16] + (crk[u] & 0xffff);
          clist[dst] = (unsigned short)q;
          float4 t = tp[q];
          if constexpr (D == 2 && SCAN_CELL_VZ) t.z = tv[q].w;     // 2-D: the speed in the unused z
          if constexpr (D == 3 && SCAN_CELL_VZ)   // 3-D: id (16 bits) | speed rounded up to bf16
            t.w = __uint_as_float((unsigned)(__float_as_int(t.w) & 0xffff) |
                                  ((__float_as_uint(tv[q].w) + 0xffffu) & 0xffff0000u));
          ctp[dst] = t;
        }
      }
      __syncthreads();
    }
  }
  stamp(1);
  // LPA lanes per agent: lane (r, h) owns curve position base + r and scans candidate slots
  // (SCH/LPA)h.. of every chunk; the partial lists are merged at the end (LPA x the waves of a
  // lane-per-agent layout, 1/LPA of the per-chunk work per lane).
  const int wave = threadIdx.x / WAVE, lane = threadIdx.x & 63, r = lane % APW, h = lane / APW;
  const int pos = bx * SCAN_AG + wave * APW + r;              // my position on the curve
  float4 me = make_float4(0.f, 0.f, 0.f, 0.f), mv = make_float4(0.f, 0.f, 0.f, 0.f);
  int i = -1;
  if (pos < Nn) {
    me = tp[pos];
    mv = tv[pos];
    i = __float_as_int(me.w);
  }
  const bool act = pos < Nn && i >= 0 && i < N;                // agents are centres, obstacles not
  const float rc = sqrtf(a.r2_check);
  // per-pair pre-test of the safety check: dangerous => |p| < r + ttc*|v_i - v_j| <= r + ttc*(|v_i|+|v_j|)
  const float base_i = rc + a.ttc_check * mv.w;
  uint64_t bk[K];
#pragma unroll
  for (int q = 0; q < K; ++q) bk[q] = KEY_EMPTY;
  bool danger = false;
  const float wminx = wave_min(act ? me.x : INFINITY), wmaxx = wave_max(act ? me.x : -INFINITY);
  const float wminy = wave_min(act ? me.y : INFINITY), wmaxy = wave_max(act ? me.y : -INFINITY);
  float wminz = 0.f, wmaxz = 0.f;
  if constexpr (D == 3) {
    wminz = wave_min(act ? me.z : INFINITY);
    wmaxz = wave_max(act ? me.z : -INFINITY);
  }
  // Temporal bound: the previous step's K neighbours are K candidates now, so the K-th distance
  // is at most the largest of their current distances. Candidates beyond it are never inserted
  // and the culling threshold is tight from the first chunk (the lists are still exact: every
  // true neighbour is within the bound; ties at the bound are kept).
  float bound = INFINITY;
  if (a.do_knn && a.prev_idx) {
    float mx = act ? 0.f : INFINITY;
    if (act) {
      const int* pr = a.prev_idx + (long)b * a.pi_env + (long)i * K;
      for (int q = h; q < K; q += LPA) {
        float pj[D];
        if constexpr (GLB) {
          float vj[D];
          load_rec<D>(Sb, (unsigned)pr[q], pj, vj);
        } else {
          const float4 c = tp[pinv[pr[q]]];
          pj[0] = c.x; pj[1] = c.y;
          if constexpr (D == 3) pj[2] = c.z;
        }
        float dp[D];
        dp[0] = me.x - pj[0];
        dp[1] = me.y - pj[1];
        if constexpr (D == 3) dp[2] = me.z - pj[2];
        mx = fmaxf(mx, sqsum<D>(dp));
      }
    }
#pragma unroll
    for (int o = APW; o < WAVE; o <<= 1) mx = fmaxf(mx, grp_xor(mx, o));
    bound = mx;
  }
  const float wvmax = wave_max(act ? mv.w : 0.f);
  const bool wave_live = __any(act);
  int cc0 = (bx * SCAN_AG + wave * APW + APW / 2) / SCH;
  if (cc0 >= nch) cc0 = nch - 1;
  float thr = wave_max(act ? bound : -INFINITY);   // bound on every agent's final K-th distance
  bool all_danger = false;
  stamp(2);
  if constexpr (CELLS) {
    if (use_cells && wave_live) {
      // this agent's cell box: its bound (kNN) and safety reach, with a margin for the float
      // rounding of d2 and of the cell mapping; its rows are tabulated below
      const float Rk = sqrtf(fmaxf(bound, 0.f)) * 1.001f + 1e-5f;
      const float Rs = a.do_safety ? (1.01f * (base_i + a.ttc_check * cgrid[6]) + 1e-4f) * 1.001f + 1e-5f : 0.f;
      float R = fmaxf(Rk, Rs);
      if constexpr ((MB_DIAG & 8) != 0) R *= 0.7f;   // negative check only: a too-small box must fail the oracle tests
      bool fin = R < INFINITY && me.x == me.x && me.y == me.y;
      if constexpr (D == 3) fin = fin && me.z == me.z;
      int c0[3] = {0, 0, 0}, c1[3] = {CG - 1, CG - 1, D == 3 ? CG - 1 : 0};
      if (fin) {
        const float pc[3] = {me.x, me.y, me.z};
#pragma unroll
        for (int d = 0; d < D; ++d) {
          c0[d] = cell_coord<CG>((pc[d] - R - cgrid[d]) * cgrid[3 + d]);
          c1[d] = cell_coord<CG>((pc[d] + R - cgrid[d]) * cgrid[3 + d]);
        }
      }
      const int ny = c1[1] - c0[1] + 1, nz = c1[2] - c0[2] + 1;
      const int nrow = act ? ny * nz : 0;
      // the box's cells in rows along x: a row's cells are consecutive cell ids, so its nodes are
      // one contiguous range of the cell-ordered arrays. Each row is trimmed to the x extent the
      // sphere of radius R leaves at the row's (y, z) distance (a disc / ball instead of the box),
      // and rows beyond R are skipped; the agent's LPA lanes take every LPA-th candidate of the
      // concatenated ranges (balanced lanes, one range read per row instead of one per cell)
      float uc[3] = {0.f, 0.f, 0.f}, csz[3] = {0.f, 0.f, 0.f};
      const float R2 = fin ? R * R : INFINITY;
      {
        const float pc[3] = {me.x, me.y, me.z};
#pragma unroll
        for (int d = 0; d < D; ++d) {
          uc[d] = (pc[d] - cgrid[d]) * cgrid[3 + d];
          csz[d] = 1.f / cgrid[3 + d];
        }
      }
      // distance from the agent to cell row / layer c along axis d (the edge cells are open:
      // cell_coord clamps), less a 1e-4-cell slack for the rounding of the cell mapping
      auto gap = [&](int c, int d) {
        const float lo = c == 0 ? -INFINITY : (float)c, hi = c == CG - 1 ? INFINITY : (float)(c + 1);
        return fmaxf(0.f, fmaxf(lo - uc[d], uc[d] - hi) - 1e-4f) * csz[d];
      };
      if constexpr (ST) {                     // counters: 12 = rows in the wave's agents' boxes
        int sc = h == 0 ? nrow : 0;
#pragma unroll
        for (int o = 1; o < WAVE; o <<= 1) sc += __shfl_xor(sc, o);
        ph[12] = sc;
      }
      // row table: the agent's LPA lanes compute the ranges of SCAN_RT rows at a time (lane h rows
      // h, h + LPA, ...; a skipped row is an empty range) into the agent's LDS slots, then every
      // lane walks them in order -- the row work leaves the divergent candidate loop
      unsigned* rt = rtab + (wave * APW + r) * SCAN_RT;
      int off = 0;                                 // candidates of the rows before, mod LPA
      for (int r0 = 0; __any(r0 < nrow); r0 += SCAN_RT) {
#pragma unroll
        for (int k = h; k < SCAN_RT; k += LPA) {
          const int rr = r0 + k;
          if (rr >= nrow) break;
          unsigned pk = 0;
          {
            const int rz = D == 3 ? rr / ny : 0;
            const int cy = c0[1] + rr - rz * ny, cz = c0[2] + rz;
            float g2 = 0.f;
            {
              const float gy = gap(cy, 1);
              g2 = gy * gy;
            }
            if constexpr (D == 3) {
              const float gz = gap(cz, 2);
              g2 += gz * gz;
            }
            if (!(g2 > R2)) {
              int x0 = c0[0], x1 = c1[0];
              if (fin) {
                // +1e-6 R^2: the cancellation in R^2 - g2 (R already carries the rounding margins)
                const float rx = sqrtf(fmaxf(R2 - g2, 0.f) + 1e-6f * R2);
                x0 = cell_coord<CG>((me.x - rx - cgrid[0]) * cgrid[3]);
                x1 = cell_coord<CG>((me.x + rx - cgrid[0]) * cgrid[3]);
              }
              int rb = cy * CG;
              if constexpr (D == 3) rb += cz * CG * CG;
              pk = (unsigned)cstart[rb + x0] | ((unsigned)cstart[rb + x1 + 1] << 16);
            }
          }
          rt[k] = pk;
        }
        __builtin_amdgcn_wave_barrier();           // the wave's own LDS writes, read back in order
        const int kn = min(SCAN_RT, nrow - r0);    // this agent's rows in the batch
        int k = 0, qi = 0, qe = 0;
        while (true) {
          while (qi >= qe && k < kn) {             // this lane's next candidate in a later row
            const unsigned pk = rt[k++];
            const int s0 = (int)(pk & 0xffffu), e0 = (int)(pk >> 16);
            qi = s0 + ((h - off) & (LPA - 1));
            qe = e0;
            off = (off + e0 - s0) & (LPA - 1);
          }
        const bool has = qi < qe;
        if (!__any(has)) break;
        if constexpr (ST) { ph[9] += 1; ph[10] += __popcll(__ballot(has)); }   // steps, candidates
        if (has) {
          const int qo = qi;
          const float4 cp = ctp[qi];
          qi += LPA;
          constexpr bool PK3 = D == 3 && SCAN_CELL_VZ;
          const int j = PK3 ? (__float_as_int(cp.w) & 0xffff) : __float_as_int(cp.w);
          float dp[D];
          dp[0] = me.x - cp.x;
          dp[1] = me.y - cp.y;
          if constexpr (D == 3) dp[2] = me.z - cp.z;
          const float d2 = sqsum<D>(dp);
          const uint64_t key = knn_key(d2, (unsigned)j);
          if (d2 <= bound && key < bk[K - 1]) topk_insert<K>(bk, key);
          if (a.do_safety && !danger) {
            // the pre-test's speed from the cell-ordered record (SCAN_CELL_VZ; 3-D: rounded up, a
            // looser pre-test), the velocity record only for the candidates that pass it
            const float vw = !SCAN_CELL_VZ ? tv[clist[qo]].w
                             : D == 2   ? cp.z
                                        : __uint_as_float(__float_as_uint(cp.w) & 0xffff0000u);
            const float lim = 1.01f * (base_i + a.ttc_check * vw) + 1e-4f;
            if (d2 < lim * lim && j != i) {
              const float4 cv = tv[clist[qo]];
              float dv[D];
              dv[0] = mv.x - cv.x;
              dv[1] = mv.y - cv.y;
              if constexpr (D == 3) dv[2] = mv.z - cv.z;
              danger = ttc_danger<D>(dp, dv, a.r2_check, a.ttc_check);
            }
          }
        }
        }
        __builtin_amdgcn_wave_barrier();           // the batch's reads before the next batch's writes
      }
    }
  }
  if (wave_live && !use_cells) {
    // gap^2 (x0.999) between this wave's box and a chunk / superchunk box
    auto gap2 = [&](const float4& cl, const float4& chh) {
      const float gx = fmaxf(0.f, fmaxf(cl.x - wmaxx, wminx - chh.x));
      const float gy = fmaxf(0.f, fmaxf(cl.y - wmaxy, wminy - chh.y));
      float bd2 = gx * gx + gy * gy;
      if constexpr (D == 3) {
        const float gz = fmaxf(0.f, fmaxf(cl.z - wmaxz, wminz - chh.z));
        bd2 = bd2 + gz * gz;
      }
      return bd2 * 0.999f;
    };
    // superchunks outward from the wave's own (sc0, sc0-1, sc0+1, ...: every one exactly once),
    // chunks of a surviving superchunk in order; both culling levels are wave-uniform
    const int sc0 = cc0 / SSC;
    for (int m = 0; m < nsc; ++m) {
      const int k = (m + 1) >> 1;
      int sc = (m & 1) ? sc0 - k : sc0 + k;
      if (sc >= nsc) sc -= nsc;
      if (sc < 0) sc += nsc;
      {
        const float4 sl = sbl[sc], sh = sbh[sc];
        const float sd2 = gap2(sl, sh);
        const float slb = 1.01f * (rc + a.ttc_check * (wvmax + sl.w)) + 1e-4f;
        const bool snk = a.do_knn && !(sd2 > thr);
        const bool sns = a.do_safety && !all_danger && !(sd2 > slb * slb);
        if constexpr (ST) ph[8] += 1;
        if (!snk && !sns) continue;
      }
      const int c_end = min(sc * SSC + SSC, nch);
      for (int cur = sc * SSC; cur < c_end; ++cur) {
        const float4 cl = cbl[cur], chh = cbh[cur];
        const float bd2 = gap2(cl, chh);
        const bool nk = a.do_knn && !(bd2 > thr);
        const float lb = 1.01f * (rc + a.ttc_check * (wvmax + cl.w)) + 1e-4f;
        const bool ns = a.do_safety && !all_danger && !(bd2 > lb * lb);
        if constexpr (ST) ph[9] += 1;
        if (!nk && !ns) continue;
        if constexpr (ST) { ph[10] += 1; ph[12] += nk ? 1 : 0; ph[13] += nk ? 0 : 1; }
        // LPA <= 8: 8 / LPA candidates per lane; LPA = 16: one per lane, lanes h >= 8 idle
        constexpr int HU = SCH / LPA > 0 ? SCH / LPA : 1;
        const bool hact = LPA <= SCH || h < SCH;
        const int hoff = hact ? HU * h : 0;
        float4 c[HU];
#pragma unroll
        for (int u = 0; u < HU; ++u) c[u] = tp[cur * SCH + hoff + u];
        bool ins = false, dch = false;            // this lane's list / danger flag changed in this chunk
#pragma unroll
        for (int u = 0; u < HU; ++u) {
          const int j = __float_as_int(c[u].w);
          float dp[D];
          dp[0] = me.x - c[u].x;
          dp[1] = me.y - c[u].y;
          if constexpr (D == 3) dp[2] = me.z - c[u].z;
          const float d2 = sqsum<D>(dp);
          const uint64_t key = knn_key(d2, (unsigned)j);
          if (hact && nk && act && d2 <= bound && key < bk[K - 1]) {
            topk_insert<K>(bk, key);
            ins = true;
          }
          if (hact && ns && act && !danger) {
            const float4 cv = tv[cur * SCH + hoff + u];
            const float lim = 1.01f * (base_i + a.ttc_check * cv.w) + 1e-4f;
            if (d2 < lim * lim && j != i) {
              float dv[D];
              dv[0] = mv.x - cv.x;
              dv[1] = mv.y - cv.y;
              if constexpr (D == 3) dv[2] = mv.z - cv.z;
              danger = ttc_danger<D>(dp, dv, a.r2_check, a.ttc_check);
              dch = dch || danger;
            }
          }
        }
        // (SCAN_THR_SKIP: no list of the wave changed in this chunk -> kth and thr are unchanged)
        if constexpr (ST) ph[11] += __any(ins) ? 1 : 0;
        if (nk && __any(ins)) {
          // the merged list's K-th distance <= min of the partial lists' K-th distances
          float kth = __uint_as_float((unsigned)(bk[K - 1] >> 32));
#pragma unroll
          for (int o = APW; o < WAVE; o <<= 1) kth = fminf(kth, grp_xor(kth, o));
          thr = wave_max(act ? fminf(kth, bound) : -INFINITY);
        }
        if (ns && __any(dch)) {
          // the lane swaps must run on every lane: never inside a short-circuit '||'
          unsigned dg = danger ? 1u : 0u;
#pragma unroll
          for (int o = APW; o < WAVE; o <<= 1) dg |= grp_xoru(dg, o);
          all_danger = !__any(act && dg == 0u);
        }
      }
    }
  }
  stamp(3);
  // merge the partial lists (butterfly: every lane ends with the full list; keys are unique:
  // (d2, node id), and the partners' lists are disjoint)
  if (a.do_knn) {
#pragma unroll
    for (int o = APW; o < WAVE; o <<= 1) {
      uint64_t px[K];
#pragma unroll
      for (int q = 0; q < K; ++q) {
        const unsigned lo = grp_xoru((unsigned)bk[q], o), hi = grp_xoru((unsigned)(bk[q] >> 32), o);
        px[q] = ((uint64_t)hi << 32) | lo;
      }
      topk_merge<K>(bk, px);
    }
  }
  {
    unsigned dg = danger ? 1u : 0u;               // unconditional lane swaps (see above)
#pragma unroll
    for (int o = APW; o < WAVE; o <<= 1) dg |= grp_xoru(dg, o);
    danger = dg != 0u;
  }
  stamp(4);
  const bool own = act && h == 0;                              // one lane reports per agent
  float ndang = 0.f, nsafe_e = 0.f, safe_ag = 0.f;
  if (act && a.do_knn) {
    // every lane of the agent holds the merged list: lane h writes slots h, h + LPA, ... and
    // their train-threshold danger bits (the per-env counts are sums of 0/1: order-free)
    int* out = a.idx + (long)b * a.i_env + (long)i * K;
    uint8_t* dout = a.dang ? a.dang + (long)b * a.i_env + (long)i * K : nullptr;
    float pi[D], vi[D];
    if constexpr (GLB) {
      load_rec<D>(Sb, (unsigned)i, pi, vi);
    } else {                                  // this lane's own staged record
      pi[0] = me.x; pi[1] = me.y; vi[0] = mv.x; vi[1] = mv.y;
      if constexpr (D == 3) { pi[2] = me.z; vi[2] = mv.z; }
    }
#pragma unroll
    for (int q0 = 0; q0 < K; q0 += LPA) {
      const int q = q0 + h;
      if (q < K) {
        uint64_t key = bk[q0];                   // bk[q] (register array: selects on h)
#pragma unroll
        for (int u = 1; u < LPA; ++u)
          if (q0 + u < K) key = (h == u) ? bk[q0 + u] : key;
        // an agent whose distances are all NaN (a diverged state) finds no candidate: its unfilled
        // slots name the agent itself, so every gather downstream stays in range
        const int j = key == KEY_EMPTY ? i : (int)(unsigned)key;
        out[q] = j;
        float pj[D], vj[D], dp[D], dv[D];
        if constexpr (GLB) {
          load_rec<D>(Sb, (unsigned)j, pj, vj);
        } else {
          const int qj = pinv[j];
          const float4 cp = tp[qj], cv = tv[qj];
          pj[0] = cp.x; pj[1] = cp.y; vj[0] = cv.x; vj[1] = cv.y;
          if constexpr (D == 3) { pj[2] = cp.z; vj[2] = cv.z; }
        }
        const float eye = (j == i) ? 1.f : 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) { dp[d] = (pi[d] - pj[d]) + eye; dv[d] = vi[d] - vj[d]; }
        const bool dg = ttc_danger<D>(dp, dv, a.r2_train, a.ttc_train);
        if (dout) dout[q] = dg ? 1 : 0;
        ndang += dg ? 1.f : 0.f;
        nsafe_e += dg ? 0.f : 1.f;
      }
    }
  }
  if (own && a.do_safety) safe_ag = danger ? 0.f : 1.f;
  stamp(5);
  ndang = wave_sum(ndang);
  nsafe_e = wave_sum(nsafe_e);
  safe_ag = wave_sum(safe_ag);
  if constexpr (D == 3 ? SCAN_WAVE_ATOMIC3 : SCAN_WAVE_ATOMIC) {
    // per-wave atomics, no block barrier: a wave does not wait for the slowest wave of its block
    // (the counts are sums of 0/1 values, exact in fp32 in any order)
    if (lane == 0) {
      if (a.do_knn && a.cnt) {
        atomicAdd(a.cnt + (long)b * a.c_env + 0, ndang);
        atomicAdd(a.cnt + (long)b * a.c_env + 1, nsafe_e);
      }
      if (a.do_safety && a.safe) atomicAdd(a.safe + (long)b * a.sf_env, safe_ag);
    }
  } else {
  if (lane == 0) { red[0][wave] = ndang; red[1][wave] = nsafe_e; red[2][wave] = safe_ag; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    for (int q = 0; q < BS / WAVE; ++q) { s0 += red[0][q]; s1 += red[1][q]; s2 += red[2][q]; }
    if (a.do_knn && a.cnt) {
      atomicAdd(a.cnt + (long)b * a.c_env + 0, s0);
      atomicAdd(a.cnt + (long)b * a.c_env + 1, s1);
    }
    if (a.do_safety && a.safe) atomicAdd(a.safe + (long)b * a.sf_env, s2);
  }
  }
  stamp(6);
  if constexpr (ST) {
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < 16; ++k) a.stamps[((long)lin0 * (BS / WAVE) + wave) * 16 + k] = ph[k];
  }
}

constexpr int SCAN_LPA = 4;      // lanes per agent (A/B at 1024 x 64: 2 -> 4 lanes 65.4 -> 61.5 us per step)

constexpr int SCAN_BS_BIG = 1024;  // block size above 512 nodes per env (4 lanes/agent: 512 -> 1024, 61.5 -> 60.5 us)
// 3-D scenes: 512-thread blocks, two per CU, so one block's slow waves overlap the other block's
// (with per-wave count atomics: see SCAN_WAVE_ATOMIC3)
constexpr int SCAN_BS_BIG3 = 512;
constexpr size_t SCAN_BOX_LDS = 160 * 1024 - 1024;   // LDS budget of the culling boxes (GLB 1)

// The launch plan of one scan call (mb_scan_plan reports it, so the tests can assert which
// instantiation they exercised): block size, lanes per agent, staging mode, whether the block
// allocates the cell grid's LDS and uses it, the grid side, per-wave count atomics, the block count
// and the dynamic LDS.
struct ScanPlan { int bs, lpa, glb, cells, use_cells, cell_g, wave_atomic, blocks; long lds; };

template <int D, int BS, int LPA>
static ScanPlan plan_kdb(const ScanArgs& a) {
  ScanPlan p{};
  p.bs = BS;
  p.lpa = LPA;
  p.blocks = (a.Nn + BS / LPA - 1) / (BS / LPA) * a.B;
  p.wave_atomic = (D == 3 ? SCAN_WAVE_ATOMIC3 : SCAN_WAVE_ATOMIC) != 0;
  if (a.Nn > SCAN_MAXN) {
    const int Np = (a.Nn + SCH - 1) / SCH * SCH, nch = Np / SCH, nsc = (nch + SSC - 1) / SSC;
    p.lds = (long)2 * (nch + nsc) * 16;
    p.glb = (size_t)p.lds > SCAN_BOX_LDS ? 2 : 1;
    if (p.glb == 2) p.lds = 0;
    return p;
  }
  // the cell grid's LDS (SCAN_CELL*) only for calls that search it (a temporal bound and a kNN
  // pass: not the first step of a rollout, not the safety-only tail scans -- ADVICE r5), and only
  // when the env still fits the 160 KB with it
  p.lds = (long)scan_lds_bytes(a.Nn);
  if constexpr (cell_on<D>()) {
    if (a.prev_idx && a.do_knn) {
      const size_t lc = scan_cell_lds<D, BS>((a.Nn + SCH - 1) / SCH * SCH, BS / LPA);
      if ((size_t)p.lds + lc + 1024 <= 160 * 1024) {
        p.lds += (long)lc;
        p.cells = 1;
        p.cell_g = cell_g<D, BS>();
      }
    }
  }
  constexpr int MQ = (4096 + BS - 1) / BS;
  p.use_cells = p.cells && a.Nn <= MQ * BS;       // the kernel's use_cells condition
  return p;
}

template <int K, int D, int BS, int LPA = SCAN_LPA>
static void launch_kdb(const ScanArgs& a, hipStream_t st, ScanPlan* plan) {
  const ScanPlan p = plan_kdb<D, BS, LPA>(a);
  if (plan) {                // mb_scan_plan: report, do not launch
    *plan = p;
    return;
  }
  dim3 grid((a.Nn + BS / LPA - 1) / (BS / LPA), a.B);
  if (p.glb) {
    const int Np = (a.Nn + SCH - 1) / SCH * SCH, nch = Np / SCH;
    hipLaunchKernelGGL(scan_stage_kernel<D>, dim3((nch + STAGE_BLOCK - 1) / STAGE_BLOCK, a.B), dim3(STAGE_BLOCK), 0,
                       st, a);
    if (p.glb == 2) {                // huge envs: the boxes stay in the global workspace
      if constexpr (BS == SCAN_BS_BIG && LPA == SCAN_LPA)
        hipLaunchKernelGGL((scan_kernel<K, D, BS, LPA, 2>), grid, dim3(BS), 0, st, a);
      return;
    }
    (void)hipFuncSetAttribute((const void*)scan_kernel<K, D, BS, LPA, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds);
    hipLaunchKernelGGL((scan_kernel<K, D, BS, LPA, 1>), grid, dim3(BS), p.lds, st, a);
    return;
  }
  ScanArgs b = a;
  b.cells = p.cells;
  if constexpr (K == 12) {
    if (a.stamps) {           // diagnostics: phase clocks (scripts/stamps_scan.py)
      (void)hipFuncSetAttribute((const void*)scan_kernel<K, D, BS, LPA, 0, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds);
      hipLaunchKernelGGL((scan_kernel<K, D, BS, LPA, 0, true>), grid, dim3(BS), p.lds, st, b);
      return;
    }
  }
  (void)hipFuncSetAttribute((const void*)scan_kernel<K, D, BS, LPA, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds);
  hipLaunchKernelGGL((scan_kernel<K, D, BS, LPA, 0>), grid, dim3(BS), p.lds, st, b);
}


static int scan_num_cu() {
  static const int cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) v = 256;
    return v;
  }();
  return cus;
}

// Small scans (a strong-scaling slice: few envs) would fill only some CUs with big blocks: use
// 256-thread blocks whenever the big-block grid has fewer blocks than CUs.
template <int D>
static bool scan_small_grid(const ScanArgs& a) {
  constexpr int AG = (D == 3 ? SCAN_BS_BIG3 : SCAN_BS_BIG) / SCAN_LPA;      // agents per big block
  return (long)a.B * ((a.Nn + AG - 1) / AG) < scan_num_cu();
}

// Still fewer 256-thread blocks than CUs (e.g. 8 envs x 1024 nodes: 128 blocks): 8 lanes per
// agent (one candidate of every chunk per lane) halve the agents per block and the per-lane
// chunk work -> twice the blocks. Same keys and tie order: the merged lists are identical for
// any LPA (tests/test_gpu_forward.py forces lanes = 4 / 8 through ScanArgs.lanes).
static bool scan_lpa8(const ScanArgs& a) {
  if (a.lanes == 4 || a.lanes == 8) return a.lanes == 8;
  constexpr int AG = 256 / SCAN_LPA;
  return SCAN_LPA < 8 && (long)a.B * ((a.Nn + AG - 1) / AG) < scan_num_cu();
}

// envs whose culling boxes exceed LDS (> ~36 K nodes): the boxes are read from the workspace,
// a layout instantiated for the 1024-thread blocks only (such envs fill the CUs by themselves)
static bool scan_boxes_global(const ScanArgs& a) {
  if (a.Nn <= SCAN_MAXN) return false;
  const int Np = (a.Nn + SCH - 1) / SCH * SCH, nch = Np / SCH, nsc = (nch + SSC - 1) / SSC;
  return (size_t)2 * (nch + nsc) * 16 > SCAN_BOX_LDS;
}

// (3-D scenes at 8 lanes per agent -- 8 agents per wave, a smaller wave box in x, y -- measured
// slower in round 5: config #5 fp16 9.93 vs 9.50-9.52 ms, profiles/r5_b6/)

// (16 lanes per agent in 512-thread blocks for the slices -- twice the threads for the per-block
// staging and cell-grid build, half the candidates per lane, a fourth merge level: oracle tests
// pass, 8-env slice 2.826 / 2.829 vs 2.830 / 2.809 ms, neutral; removed, profiles/r6c/)

template <int K, int D>
static void launch_kd(const ScanArgs& a, hipStream_t st, ScanPlan* plan) {
  if (scan_boxes_global(a)) launch_kdb<K, D, SCAN_BS_BIG>(a, st, plan);
  else if (scan_lpa8(a)) launch_kdb<K, D, 256, 8>(a, st, plan);
  else if (a.Nn > 512 && !scan_small_grid<D>(a)) launch_kdb<K, D, D == 3 ? SCAN_BS_BIG3 : SCAN_BS_BIG>(a, st, plan);
  else launch_kdb<K, D, 256>(a, st, plan);
}

template <int K>
static void launch_k(const ScanArgs& a, hipStream_t st, ScanPlan* plan = nullptr) {
  if (a.dim == 3) launch_kd<K, 3>(a, st, plan);
  else launch_kd<K, 2>(a, st, plan);
}

}  // namespace mb

extern "C" int mb_cell_sort(const mb::CellSortArgs* a, hipStream_t st) {
  using namespace mb;
  hipLaunchKernelGGL(cell_sort_kernel, dim3(a->B), dim3(SORT_BLOCK), 0, st, *a);
  return (int)hipGetLastError();
}

extern "C" int mb_scan(const mb::ScanArgs* a, hipStream_t st) {
  using namespace mb;
  if (a->Nn < a->N || !a->perm) return -3;
  if (a->Nn > SCAN_MAXN) {       // global staging: the workspace must hold scan_ws_f4(Nn) per env
    const int Np = (a->Nn + SCH - 1) / SCH * SCH, nch = Np / SCH, nsc = (nch + SSC - 1) / SSC;
    if (!a->ws || a->ws_env < 2L * Np + 2L * (nch + nsc)) return -4;
  }
  switch (a->do_knn ? a->K : 1) {
#define CASE(k) case k: launch_k<k>(*a, st); break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
    CASE(9) CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16)
#undef CASE
    default: return -1;
  }
  return (int)hipGetLastError();
}

// The plan mb_scan would launch for these arguments (no launch; the plan does not depend on K):
// out = {block size, lanes per agent, staging mode (0 LDS, 1 global records, 2 global boxes),
// cell LDS allocated, cell grid searched, cell grid side, per-wave count atomics, blocks, LDS bytes}
extern "C" int mb_scan_plan(const mb::ScanArgs* a, long* out) {
  using namespace mb;
  if (a->Nn < a->N) return -3;
  ScanPlan p{};
  launch_k<1>(*a, nullptr, &p);
  const long v[9] = {p.bs, p.lpa, p.glb, p.cells, p.use_cells, p.cell_g, p.wave_atomic, p.blocks, p.lds};
  for (int k = 0; k < 9; ++k) out[k] = v[k];
  return 0;
}
