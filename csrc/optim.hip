// Optimizer-side kernels, gfx950: deterministic reduction of per-workgroup weight-gradient
// slabs, and the fused flat Adam (torch.optim.Adam semantics, L2 weight decay) over one
// contiguous parameter range -- the two reference optimizers (train.py:36-37) are two ranges
// of the single flat fp32 master buffer.
#include "common.h"
#include "args.h"

namespace mb {

// out[c] (+)= sum_r partial[r * cols + c] in a fixed order (bitwise reproducible).
// Block = 16 float4-column groups x 16 row slices: slice y sums rows y, y+16, ... in order, then
// the 16 slice sums are added in slice order through LDS. ~300 workgroups for the CBF slab
// instead of 19 with one serial thread per column.
constexpr int RR_COLS = 16, RR_SLICES = 16;
DEV void reduce_rows_block(const float* partial, int rows, int cols, float* out, int accumulate, int bx) {
  __shared__ float4 red[RR_SLICES][RR_COLS];
  const int cx = threadIdx.x % RR_COLS, sy = threadIdx.x / RR_COLS;
  const int c4 = bx * RR_COLS + cx;
  const bool ok = c4 * 4 < cols;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok) {
    // 8 rows' loads in flight before their (in-order) adds: the slabs come from HBM / MALL, and
    // one dependent round trip per 4 rows made the reduction latency-bound (~1 TB/s)
    for (int r = sy; r < rows; r += 8 * RR_SLICES) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int rr = min(r + u * RR_SLICES, rows - 1);
        v[u] = *reinterpret_cast<const float4*>(partial + (long)rr * cols + c4 * 4);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (r + u * RR_SLICES < rows) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
    }
  }
  red[sy][cx] = s;
  __syncthreads();
  if (sy == 0 && ok) {
    float4 t = red[0][cx];
    for (int y = 1; y < RR_SLICES; ++y) {
      const float4 v = red[y][cx];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    float4* o = reinterpret_cast<float4*>(out + c4 * 4);
    if (accumulate) {
      const float4 p = *o;
      t.x += p.x; t.y += p.y; t.z += p.z; t.w += p.w;
    }
    *o = t;
  }
}

// Narrow slabs (<= 16 columns: the CBF loss partials, 12 floats x 16 rows per CU): one block, 64 row
// slices x 4 column groups -- the wide layout's 16 slices left each thread 1/16 of thousands of rows
// in a dependent chain, the iteration's slowest block
constexpr int RN_SLICES = RR_COLS * RR_SLICES / 4;
DEV void reduce_rows_narrow(const float* partial, int rows, int cols, float* out, int accumulate) {
  __shared__ float4 redn[RN_SLICES][4];
  const int cx = threadIdx.x % 4, sy = threadIdx.x / 4;
  const bool ok = cx * 4 < cols;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok) {
    for (int r = sy; r < rows; r += 8 * RN_SLICES) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int rr = min(r + u * RN_SLICES, rows - 1);
        v[u] = *reinterpret_cast<const float4*>(partial + (long)rr * cols + cx * 4);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (r + u * RN_SLICES < rows) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
    }
  }
  redn[sy][cx] = s;
  __syncthreads();
  if (sy == 0 && ok) {
    float4 t = redn[0][cx];
    for (int y = 1; y < RN_SLICES; ++y) {
      const float4 v = redn[y][cx];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    float4* o = reinterpret_cast<float4*>(out + cx * 4);
    if (accumulate) {
      const float4 p = *o;
      t.x += p.x; t.y += p.y; t.z += p.z; t.w += p.w;
    }
    *o = t;
  }
}

__global__ __launch_bounds__(RR_COLS * RR_SLICES) void reduce_rows_kernel(const float* partial, int rows, int cols,
                                                                          float* out, int accumulate) {
  if (cols <= 16) reduce_rows_narrow(partial, rows, cols, out, accumulate);
  else reduce_rows_block(partial, rows, cols, out, accumulate, blockIdx.x);
}

// Several independent slab reductions in ONE launch (the CBF, node and edge weight-gradient slabs
// and the loss partials after the backward): job j owns blocks [blk0[j], blk0[j + 1]), each block
// the same fixed-order column-group reduction as reduce_rows_kernel (bitwise the same sums)
__global__ __launch_bounds__(RR_COLS * RR_SLICES) void reduce_multi_kernel(ReduceMultiArgs a) {
  int j = 0;
  while (j + 1 < a.njobs && (int)blockIdx.x >= a.blk0[j + 1]) ++j;
  if (a.cols[j] <= 16) reduce_rows_narrow(a.partial[j], a.rows[j], a.cols[j], a.out[j], a.accumulate[j]);
  else reduce_rows_block(a.partial[j], a.rows[j], a.cols[j], a.out[j], a.accumulate[j], (int)blockIdx.x - a.blk0[j]);
}

DEV void adam_block(const AdamArgs& a, int bx) {
  const int i = a.lo + bx * blockDim.x + threadIdx.x;
  if (i >= a.hi) return;
  // device-side failure guard: a non-finite reduced gradient skips the whole step (the flag is
  // the same on every rank after the all-reduce), with no host round trip
  if (a.ok && *a.ok == 0) return;
  float step_size = a.step_size, bc2_sqrt = a.bc2_sqrt;
  if (a.step) {   // bias corrections of step t = *step + 1 (torch.optim.Adam, in double)
    const double t = (double)(*a.step + 1);
    step_size = (float)((double)a.lr / (1.0 - pow((double)a.b1, t)));
    bc2_sqrt = (float)sqrt(1.0 - pow((double)a.b2, t));
  }
  float g = a.grad[i];
  float p = a.param[i];
  if (a.wd != 0.f) g = g + a.wd * p;
  float m = a.m[i], v = a.v[i];
  m = a.b1 * m + (1.f - a.b1) * g;
  v = a.b2 * v + (1.f - a.b2) * g * g;
  a.m[i] = m;
  a.v[i] = v;
  const float denom = sqrtf(v) / bc2_sqrt + a.eps;
  a.param[i] = p - step_size * (m / denom);
}

__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) { adam_block(a, blockIdx.x); }

// The Adam steps of several parameter groups (the two reference optimizers, train.py:36-37) in
// ONE launch: group g owns blocks [blk0[g], blk0[g + 1]); same per-element arithmetic
__global__ __launch_bounds__(256) void adam_multi_kernel(AdamMultiArgs a) {
  int g = 0;
  while (g + 1 < a.ngroups && (int)blockIdx.x >= a.blk0[g + 1]) ++g;
  adam_block(a.g[g], (int)blockIdx.x - a.blk0[g]);
}

// Weight repacking after an optimizer step: every MFMA fragment / row-major image / side vector
// of both networks is a gather of the flat fp32 master parameters (index maps from
// ops/layout.py; index n = constant 0, n + 1 = constant 1), in ONE launch: 16-bit outputs
// (bf16 RNE or fp16) then fp32 outputs.
DEV void step_commit_body(const StepCommitArgs& a);
// commit (optional): the optimizer step's commit (step_commit_kernel's work) by one thread -- the
// gather runs after the Adam launch, whose reads of the step counters and the guard flag are then
// complete (kernel boundary): one launch fewer per iteration
__global__ __launch_bounds__(256) void pack_gather_kernel(const float* src, int n, const int* idx16, int m16,
                                                          unsigned short* out16, int f16, const int* idx32, int m32,
                                                          float* out32, StepCommitArgs commit) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (commit.ok && i == 0) step_commit_body(commit);
  if (i < m16) {
    // bit 30 of an index selects the bf16 residual v - bf16(v) (the lo plane of the x3 split)
    const int k0 = idx16[i];
    const int k = k0 & 0x3FFFFFFF;
    const float v = k < n ? src[k] : (k == n ? 0.f : 1.f);
    unsigned short hbits;
    if (f16) {
      const _Float16 hv = (_Float16)v;
      hbits = __builtin_bit_cast(unsigned short, hv);
    } else {
      const __bf16 hi = (__bf16)v;                     // round to nearest even
      const __bf16 bv = (k0 & 0x40000000) ? (__bf16)(v - (float)hi) : hi;
      hbits = __builtin_bit_cast(unsigned short, bv);
    }
    out16[i] = hbits;
  } else if (i < m16 + m32) {
    const int k = idx32[i - m16];
    out32[i - m16] = k < n ? src[k] : (k == n ? 0.f : 1.f);
  }
}

// Flat gradient assembly: grad[p] = scale * sum of the reduced slab entries that map to
// parameter p (CSR by p, fixed order: deterministic, no atomics, no zero-fill)
// Optional in the same launch (single-process runs: no all-reduce follows): ok <- 0 if any assembled
// element is not finite (grad_check_kernel's test), and one extra block writes the iteration's
// statistics row (stats_pack_kernel's work) -- two launches fewer per iteration
DEV void stats_pack_body(const float* sums, const float* counts, const float* local, float* row, int t);
__global__ __launch_bounds__(256) void grad_assemble_kernel(GradAssembleArgs a) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (a.row && (int)blockIdx.x == (a.n + 255) / 256) {
    stats_pack_body(a.sums, a.counts, a.local, a.row, threadIdx.x);
    return;
  }
  float scale = a.scale;
  if (a.gscale) scale /= *a.gscale;     // fp16: unscale by the device loss scale
  bool bad = false;
  if (p < a.n) {
    float t = 0.f;
    for (int q = a.ptr[p]; q < a.ptr[p + 1]; ++q) t += a.red[a.src[q]];
    const float v = t * scale;
    a.grad[p] = v;
    bad = !isfinite(v);
  }
  if (a.ok && __any(bad) && (threadIdx.x % WAVE) == 0) *a.ok = 0;
}

// ok = 0 if any gradient element is not finite (ok is 1 between steps: step_commit resets it)
__global__ __launch_bounds__(256) void grad_check_kernel(const float* g, int n, int* ok) {
  bool bad = false;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) bad = bad || !isfinite(g[i]);
  if (__any(bad) && (threadIdx.x % WAVE) == 0) *ok = 0;
}

// after the Adam launches of one iteration (see StepCommitArgs): no host round trip, no
// torch glue kernels between the optimizer and the next iteration
DEV void step_commit_body(const StepCommitArgs& a) {
  const int ok = *a.ok;
  if (ok) {
    for (int g = 0; g < a.ngroups; ++g)
      if ((a.mask >> g) & 1) a.steps[g] += 1;
  } else {
    *a.skipped += 1;
  }
  if (a.gscale) {
    float s = *a.gscale;
    if (!ok) {
      s = fmaxf(0.5f * s, 1.f);
      *a.good = 0;
    } else {
      const int g = *a.good + 1;
      if (g >= a.growth) {
        s = fminf(2.f * s, a.max_scale);
        *a.good = 0;
      } else {
        *a.good = g;
      }
    }
    *a.gscale = s;
  }
  if (a.stats_row) {
    if (a.stats_src)
      for (int q = 0; q < 16; ++q) a.stats_row[q] = a.stats_src[q];
    a.stats_row[16] = ok ? 0.f : 1.f;
    a.stats_row[17] = a.gscale ? *a.gscale : 1.f;
  }
  *a.ok = 1;
}

__global__ void step_commit_kernel(StepCommitArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  step_commit_body(a);
}

// One iteration's statistics row (utils.metrics.StepStats): [10 loss sums | counts 3 | local 3 |
// skipped | loss scale] -- written into a ring of rows instead of torch.cat + clone
__global__ void stats_pack_kernel(const float* sums, const float* counts, const float* local, float* row) {
  stats_pack_body(sums, counts, local, row, threadIdx.x);
}
DEV void stats_pack_body(const float* sums, const float* counts, const float* local, float* row, int t) {
  if (t < 10) row[t] = sums[t];
  else if (t < 13) row[t] = counts[t - 10];
  else if (t < 16) row[t] = local[t - 13];
  else if (t < 18) row[t] = t == 16 ? 0.f : 1.f;
}

// Post-rollout bookkeeping in one launch (replaces ~20 small tensor ops between the rollout
// and the backward). Env b's step t is valid iff the env was not done before t, done after
// step t meaning dist[t, b] / N < thr (train.py:78-81 with per-env masks). Outputs the (T, B)
// validity mask, the pooled counts [n_dang, n_safe, n_act] of this rank (all-reduced by the
// caller) and the local stats [agent-steps, safe agents of s_{t+1}, action-loss sum]. One
// block, fixed-order reduction: deterministic.
constexpr int RS_BLOCK = 256;
__global__ __launch_bounds__(RS_BLOCK) void rollout_stats_kernel(RolloutStatsArgs a) {
  float v[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // the step records of RS_T steps are requested together (clamped, unconditional), then consumed
  // in step order: one memory round trip per RS_T steps instead of one per step (the per-env
  // chain was ~30 us at the headline, on the critical path between the rollout and the backward)
  constexpr int RS_T = 8;
  for (int b = threadIdx.x; b < a.B; b += RS_BLOCK) {
    bool done = false;
    for (int t0 = 0; t0 < a.T; t0 += RS_T) {
      float c0[RS_T], c1[RS_T], sf[RS_T];
      unsigned long long dq[RS_T], aq[RS_T];
#pragma unroll
      for (int u = 0; u < RS_T; ++u) {
        const int t = min(t0 + u, a.T - 1);
        c0[u] = a.cnt[(t * a.B + b) * 2];
        c1[u] = a.cnt[(t * a.B + b) * 2 + 1];
        sf[u] = a.safe ? a.safe[(t + 1) * a.B + b] : 0.f;
        aq[u] = a.act ? a.act[t * a.B + b] : 0ull;
        dq[u] = a.dist[t * a.B + b];
      }
#pragma unroll
      for (int u = 0; u < RS_T; ++u) {
        const int t = t0 + u;
        if (t >= a.T) break;
        const bool vl = !done;
        a.valid[t * a.B + b] = vl ? 1 : 0;
        if (vl) {
          v[0] += c0[u];
          v[1] += c1[u];
          v[2] += (float)a.N;
          if (a.safe) v[3] += sf[u];
          if (a.act)     // a saturated (diverged) agent term: the action loss is not a number
            v[4] += (double)aq[u] >= FX_SAT ? __builtin_nanf("") : (float)((double)aq[u] / FX_ACT);
        }
        done = done || ((float)((double)dq[u] / FX_DIST) / (float)a.N < a.thr);
      }
    }
  }
  __shared__ float red[6][RS_BLOCK];
#pragma unroll
  for (int q = 0; q < 5; ++q) red[q][threadIdx.x] = v[q];
  __syncthreads();
  for (int o = RS_BLOCK / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o)
#pragma unroll
      for (int q = 0; q < 5; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.counts[0] = red[0][0];
    a.counts[1] = red[1][0];
    a.counts[2] = red[2][0];
    a.local[0] = red[2][0];
    a.local[1] = red[3][0];
    a.local[2] = red[4][0];
  }
  if (a.reset_T > 0) {     // every read above precedes the reduction's barriers
    const int n = a.reset_T * a.B;
    for (int q = threadIdx.x; q < n; q += RS_BLOCK) {
      a.dist[q] = 0ull;
      a.cnt[2 * q] = 0.f;
      a.cnt[2 * q + 1] = 0.f;
      if (a.act) a.act[q] = 0ull;
    }
    if (a.safe)
      for (int q = threadIdx.x; q < n + a.B; q += RS_BLOCK) a.safe[q] = 0.f;
  }
}

}  // namespace mb

extern "C" int mb_pack_gather(const float* src, int n, const int* idx16, int m16, unsigned short* out16, int f16,
                              const int* idx32, int m32, float* out32, const mb::StepCommitArgs* commit,
                              hipStream_t st) {
  using namespace mb;
  const int tot = m16 + m32;
  StepCommitArgs c{};
  if (commit) c = *commit;
  hipLaunchKernelGGL(pack_gather_kernel, dim3(tot > 0 ? (tot + 255) / 256 : 1), dim3(256), 0, st, src, n, idx16, m16,
                     out16, f16, idx32, m32, out32, c);
  return (int)hipGetLastError();
}

extern "C" int mb_grad_assemble(const mb::GradAssembleArgs* a, hipStream_t st) {
  using namespace mb;
  const int blocks = (a->n + 255) / 256 + (a->row ? 1 : 0);
  hipLaunchKernelGGL(grad_assemble_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, *a);
  return (int)hipGetLastError();
}

extern "C" int mb_reduce_multi(const mb::ReduceMultiArgs* a, hipStream_t st) {
  using namespace mb;
  if (a->njobs < 1 || a->njobs > RM_JOBS) return -1;
  ReduceMultiArgs b = *a;
  int blk = 0;
  for (int j = 0; j < b.njobs; ++j) {
    if (b.cols[j] % 4) return -1;
    b.blk0[j] = blk;
    blk += (b.cols[j] / 4 + RR_COLS - 1) / RR_COLS;
  }
  hipLaunchKernelGGL(reduce_multi_kernel, dim3(blk), dim3(RR_COLS * RR_SLICES), 0, st, b);
  return (int)hipGetLastError();
}

extern "C" int mb_adam_multi(const mb::AdamMultiArgs* a, hipStream_t st) {
  using namespace mb;
  if (a->ngroups < 1 || a->ngroups > AM_GROUPS) return -1;
  AdamMultiArgs b = *a;
  int blk = 0;
  for (int g = 0; g < b.ngroups; ++g) {
    b.blk0[g] = blk;
    const int n = b.g[g].hi - b.g[g].lo;
    blk += n > 0 ? (n + 255) / 256 : 0;
  }
  if (blk == 0) return 0;
  hipLaunchKernelGGL(adam_multi_kernel, dim3(blk), dim3(256), 0, st, b);
  return (int)hipGetLastError();
}

extern "C" int mb_grad_check(const float* g, int n, int* ok, hipStream_t st) {
  using namespace mb;
  const int blocks = (n + 255) / 256 < 256 ? (n + 255) / 256 : 256;
  hipLaunchKernelGGL(grad_check_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, g, n, ok);
  return (int)hipGetLastError();
}

extern "C" int mb_step_commit(const mb::StepCommitArgs* a, hipStream_t st) {
  using namespace mb;
  hipLaunchKernelGGL(step_commit_kernel, dim3(1), dim3(64), 0, st, *a);
  return (int)hipGetLastError();
}

extern "C" int mb_stats_pack(const float* sums, const float* counts, const float* local, float* row, hipStream_t st) {
  using namespace mb;
  hipLaunchKernelGGL(stats_pack_kernel, dim3(1), dim3(64), 0, st, sums, counts, local, row);
  return (int)hipGetLastError();
}

extern "C" int mb_rollout_stats(const mb::RolloutStatsArgs* a, hipStream_t st) {
  using namespace mb;
  hipLaunchKernelGGL(rollout_stats_kernel, dim3(1), dim3(RS_BLOCK), 0, st, *a);
  return (int)hipGetLastError();
}

extern "C" int mb_reduce_rows(const float* partial, int rows, int cols, float* out, int accumulate, hipStream_t st) {
  if (cols % 4) return -1;
  const int groups = cols / 4;
  hipLaunchKernelGGL(mb::reduce_rows_kernel, dim3((groups + mb::RR_COLS - 1) / mb::RR_COLS),
                     dim3(mb::RR_COLS * mb::RR_SLICES), 0, st, partial, rows, cols, out, accumulate);
  return (int)hipGetLastError();
}

extern "C" int mb_adam(const mb::AdamArgs* a, hipStream_t st) {
  const int n = a->hi - a->lo;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(mb::adam_kernel, dim3((n + 255) / 256), dim3(256), 0, st, *a);
  return (int)hipGetLastError();
}
