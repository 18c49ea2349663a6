// Kernel argument structs shared by the HIP sources and the pybind11 layer.
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "prec.h"

namespace mb {

// Per-env rollout sums (goal distance, action-loss term) are accumulated as fixed-point 64-bit
// integers: integer atomics commute, so the sums -- and the early-stop horizon that depends on
// them -- do not depend on the order in which waves finish. value = sum / FX_*.
constexpr double FX_DIST = 4294967296.0;   // 2^32: per-env distance sums < 2^31 for any env size here
constexpr double FX_ACT = 16777216.0;      // 2^24: per-env action-term sums < 2^39
// per-agent saturation of the fixed-point terms: a non-finite (diverged) or absurdly large term
// becomes 2^46 (a goal distance of 2^14), so its env never looks done (mean >= 2^14 / N > 0.07 for
// any N here) and an action sum >= FX_SAT is reported as NaN; 2^17 saturated agents fit an int64
constexpr double FX_SAT = 70368744177664.0;   // 2^46

struct CellSortArgs {
  const float4* S;  long s_env;      // node (b,i) record at S[(b*s_env + i) * rec]
  int B, N;                          // N = graph nodes (agents + obstacle points)
  int rec;                           // float4s per node record (1: 2-D, 2: 3-D)
  float L;                           // scenario side length (curve grid spans [0, L]^2)
  int* perm;                         // (B, N) position on the curve -> agent id
};

struct ScanArgs {
  const float4* S;  long s_env;      // node (b,i) record at S[(b*s_env + i) * REC<dim>]
  const int* perm;                   // (B, Nn) Hilbert order from cell_sort
  int B, N, K;                       // N agents (centres; the first N nodes)
  int Nn;                            // graph nodes: agents + static obstacle points
  int dim;
  int* idx;         long i_env;      // (b,i,k) at idx[b*i_env + i*K + k]
  uint8_t* dang;                     // same indexing as idx (may be null)
  float* cnt;       long c_env;      // cnt[b*c_env + {0: dangerous edges, 1: safe edges}]
  float* safe;      long sf_env;     // safe[b*sf_env] += #agents with no dangerous pair
  float r2_train, ttc_train, r2_check, ttc_check;
  int do_knn, do_safety;
  const int* prev_idx; long pi_env;  // previous step's kNN (b,i,k) (or null): temporal K-th bound
  float4* ws; long ws_env;           // Nn > 4096: per-env global staging (float4s per env), else null
  int lanes;                         // lanes per agent: 0 = by grid size (scan.hip scan_lpa8), 4 or 8
  unsigned long long* stamps;        // diagnostics: phase clocks [block][wave][16] (K = 12 LDS path; null = off)
  int cells;                         // set by the launcher: the cell-grid LDS was allocated (scan.hip SCAN_CELL*)
};

struct ScenArgs {
  float4* S;      long s_env;     // node records out (agents only; velocity 0), strides in records
  float* G;       // (B, N, D) goals out
  const float* obs; int M;        // (B, M, D) static obstacle points (conflict points) or M = 0
  int dim;
  int B, N;
  float L, r, spread;
  unsigned long long seed;
  int max_rounds;
  int* status;    // per env: rounds used for goals (or -1 if max_rounds hit)
  unsigned char* ws; long ws_env;   // envs too large for LDS: per-env global workspace (bytes), else null
};

struct CtrlArgs {
  const float4* S;  long s_env;       // node records at step t: (b,i) -> S[(b*s_env + i) * REC]
  int dim;                            // 2 or 3; vectors below hold D floats per agent
  const float* G;                     // goals (b,i,d) -> G[(b*N + i)*D + d]
  const int* idx;   long i_env;       // (b,i,k) -> idx[b*i_env + i*K + k]
  int B, N, K;
  const h16* wpack;                  // packed ctrl fragments
  int f_edge;                         // fragment offset of ew1f (ew2 follows)
  int f_node;                         // fragment offset of nw1f (nw2, nw3, nw4 follow)
  const float* wvec;                  // eb2|nb2|nb3|nb4 (CTRL_VEC floats)
  float* A;         long a_env;       // actions out (b,i,d) -> A[(b*a_env + i)*D + d] (may be null)
  float4* Snext;    long sn_env;      // next-state records out (may be null)
  unsigned long long* dist_sum; long d_env;  // per-env sum of |p' - g| * FX_DIST (may be null)
  unsigned long long* act_sum;  long ac_env; // per-env sum of |‖a‖² - ‖a_ref‖²| * FX_ACT (may be null)
  const float* noise; long n_env;     // additive action noise (b,i,d) (may be null)
  // device-side exploration noise (reference train.py:65-67): with probability noise_prob per
  // (env, step) every agent's action gets noise_scale * N(0, 1); counter-based RNG keyed by the
  // per-iteration key *noise_key (seed, iteration, rank), the step noise_t, env, agent, axis.
  const unsigned long long* noise_key; // device scalar or null (no noise)
  float noise_prob, noise_scale;
  int noise_t;
  float dt, obs_r, sqrt3;
  h16* pooled;     long p_env;       // (b,i,128) max-pooled edge features out (h16), or null
  uint8_t* argmax;  long am_env;      // (b,i,128) winning slot per feature (0xFF: no grad), or null
  int apw;                            // agents per wave (even, 2..32; 0 = 32): small scenes use fewer
  int b0, nb_total;                   // env offset / total envs of a per-env view (noise keys; 0, 0 = this view)
  // early-stop publication (native rollout driver; null = off): the step's last workgroup copies
  // the B per-env dist_sum values to host-coherent pub_dist and then stores pub_gen to *pub_flag
  unsigned* pub_ctr;                  // this step's workgroup counter (zeroed before the rollout)
  unsigned long long* pub_dist;       // host-coherent (B) slots of this step
  unsigned* pub_flag;                 // host-coherent flag of this step
  unsigned pub_gen;                   // the rollout's generation number
  unsigned long long* stamps;         // diagnostics: phase clocks [block][wave][16] (x3 step; null = off)
  // the node MLP's activations out, for the cooperative node backward to reuse instead of
  // recomputing them: agent (b,i) -> acts + (b*na_env + i) * NODE_ACT_BYTES (ctrl.hip), or null
  unsigned char* acts; long na_env;
};

// Persistent small-scene rollout (ctrl.hip rollout_small_kernel): one workgroup per env runs
// every step of the rollout in one launch.
struct RolloutSmallArgs {
  CtrlArgs c;           // time-major bases: S (T+1,B,Nn), A (T,B,N), dist/act sums (T,B), pooled,
                        // argmax (T,B,N,.); weights, noise and constants as for one step
  int* idx;             // (>=T, B, N, K) kNN out (row Tmax only with knn_tail)
  uint8_t* dang;        // (T, B, N, K)
  float* cnt;           // (T, B, 2)
  float* safe;          // (T+1, B) or null (no safety statistic)
  int Nn, Tmax, knn_tail;
  float r2_train, ttc_train, r2_check, ttc_check;
  float done_thr;       // early stop: mean goal distance < done_thr (-inf: run all Tmax steps)
  int* ctl;             // [envs done, max first-done step, finished workgroups]: zero at the launch
                        // (with res: re-armed by the kernel's last workgroup)
  int* res;             // optional host-coherent [T, flag]: the horizon, then flag = res_gen
  int res_gen;
  const float* s0;      // optional (B, N, 2D) start states: written into the S[0] records first
  const float* g0;      // optional (B, N, D) goals: copied into c.G first
};

struct LossConsts {
  float eps_dang, dt_alpha, w_dang, w_safe, w_dang_d, w_safe_d, scale;
  const float* gscale;        // optional device loss scale (fp16 dynamic scaling): multiplies `scale`
};
// upstream-gradient multiplier of the hinge terms (the device loss scale folded in)
__host__ __device__ inline float lc_scale(const LossConsts& lc) { return lc.gscale ? lc.scale * *lc.gscale : lc.scale; }

struct CbfFwdArgs {
  const float4* S;  long s_env, s_step;   // node record of (b,t,i): S[(b*s_env + t*s_step + i) * REC]
  int dim;                                 // 2 or 3
  const int* idx;                          // (T,B,N,K) contiguous (time-major)
  const uint8_t* dang;                     // (T,B,N,K) or null (all safe)
  const uint8_t* valid;                    // (T,B) or null (all valid)
  int B, T, N, K;
  int two;                                 // also evaluate h' on s_{t+1}
  const h16* wpack; int f_fwd;            // fragment offset of w1f (w2, w3 follow)
  const float* wvec;
  float* h_out;                            // (E) or null
  float* hn_out;                           // (E) or null
  float* dh_out;                           // (2,E) or null: [dL/dh ; dL/dh']
  const float* counts;                     // device [n_dang, n_safe] (global) for dh
  float* partial;                          // (gridDim.x, 10) or null
  LossConsts lc;
  float obs_r, dist_thr, dist_eps;
  // deduplicated evaluation list (src != null; see dedup.hip): evaluation u < *nev, u < E is the
  // main slot u on s_t, u >= E an extra evaluation of slot src[u] on s_{t+1} (neighbour from
  // idx1); h_out[u] = masked h, mask_out[u] = radius mask
  const int* src;
  const int* nev;
  const int* idx1;
  uint8_t* mask_out;
  const h16* wrm;                          // row-major W2 | W3 images (dedup forward)
  // dedup forward range: evaluations u_begin <= u < (u_end ? u_end : *nev). Main-slot slices of
  // one rollout step run during the rollout (T = t+1 there, so every u < E is a main slot).
  unsigned u_begin, u_end;
};

struct CbfBwdArgs {
  const float4* S;  long s_env, s_step;   // node record of (b,t,i): S[(b*s_env + t*s_step + i) * REC]
  int dim;                                 // 2 or 3
  const int* idx;                          // (T,B,N,K) time-major
  const int* idx1;                         // neighbour slots of pass 1 (null = idx: reuse_nbr_idx)
  int B, T, N, K;
  int passes;                              // evaluations = passes*E; pass p reads states at t+p
  const float* dh;                         // (passes, E) upstream dL/dh (radius mask folded in)
  const h16* wpack; int f_bwd;            // fragment offset of w1f (w2,w3,w3t,w2t,w1ft follow)
  const h16* wrm;                         // row-major W2 [128][72] | W3 [64][136] images
  const float* wvec;
  float4* dE;                              // (passes, E) records of dL/d(s_i - s_j), or null
  float* partial;                          // (gridDim.x, CBF_PARTIAL) per-workgroup dW slabs
  float obs_r, dist_thr, dist_eps;
  // fused training mode (passes == 2): dh is computed in-kernel from h(s_t), h'(s_{t+1}) of the
  // same edge, the danger bit, env-step validity and the global pooled counts; the 10 loss
  // partial sums go to the slab at P_LOSS (dh is then not read)
  int fused;
  const uint8_t* dang;                     // (T,B,N,K)
  const uint8_t* valid;                    // (T,B) or null
  const float* counts;                     // [n_dang, n_safe] global
  LossConsts lc;
  // deduplicated evaluation list (non-fused; src != null): evaluations u < *nev addressed as in
  // CbfFwdArgs, dh / dE indexed by u
  const int* src;
  const int* nev;
  // active list (optional): only evaluations act[v], v < *nact, are processed (dh != 0)
  const int* act;
  const int* nact;
  // 16x16x32 x3 backward (csrc/cbf16.h; rec != null selects it): cbf_compact's 16-byte records
  // of the active evaluations, the column-permuted W2 | W3 images and the layer-1 fragments
  const int4* rec;
  const h16* wrm16;
  const h16* w16;
  float* dbg;                   // diagnostics (null in production): per-record forward sums (cbf16)
  unsigned long long* stamps;   // diagnostics (null in production): per-wave shader-clock cycles
                                // summed per phase over the wave's chunks, [workgroup][wave][8]
                                // (scripts/stamps_cbf.py)
};

// Deduplication of the h / h' evaluations (dedup.hip). h'(s_{t+1}) of slot (t,b,i,k) is the
// same function value as h(s_{t+1}) of the slot (t+1,b,i,k') with the same neighbour, so only
// the unmatched pairs ("extras") need their own evaluation.
struct CbfMatchArgs {
  const int* idx;        // (T+G1, B, N, K) neighbour slots (G1 = 1: h' on the recomputed kNN)
  int T, B, N, K;
  int mode;              // 0: reuse_nbr_idx (match by neighbour id), 1: recomputed kNN (slot k <-> k)
  int phase;             // 0: match, counts, map1 / src except the extras' offsets; 1: the extras' offsets
  int* cnt;              // (T*B*N) extras per (t,b,i) row (phase 0 out, phase 1 in)
  const int* off;        // (T*B*N) exclusive offsets (phase 1 in; null: computed in-kernel from bsum)
  int* bsum;             // (gridDim.x) extras per block (phase 0 out, phase 1 in)
  int* nev;              // [E + extras] (phase 1 out, written by the last block)
  int* map1;             // (E) evaluation index of the h' partner of main slot e (phase 0 null: counts only)
  int* src;              // (2E) source slot whose h' is evaluation u, or -1
};

struct CbfDhArgs {
  const float* h;        // (U) masked h per evaluation
  const uint8_t* hmask;  // (U) radius mask per evaluation
  const int* map1; const int* src; const int* nev;
  const uint8_t* dang;   // (T,B,N,K)
  const uint8_t* valid;  // (T,B) or null
  int B, T, N, K;
  const float* counts;   // [n_dang, n_safe] global
  LossConsts lc;
  float* dh;             // (U) upstream gradient per evaluation
  float* partial;        // (gridDim.x, 12) loss partial sums (slots 0..9 as CBF P_LOSS)
  int* blk_active;       // (gridDim.x) evaluations with dh != 0 per block (or null)
};

struct CtrlNodeBwdArgs {
  const h16* pooled;  long p_env;     // (b,i,128) pooled edge features of step t (rollout)
  const float4* S;     long s_env;     // node records s_t
  int dim;
  const float* G;                      // goals (B,N,D)
  const float* A;      long a_env;     // actions a_t as applied (incl. noise), D per agent
  const float4* Gn;    long gn_env;    // G_{t+1} = dL/ds_{t+1} records (or null)
  const uint8_t* valid; long v_env;    // valid[b*v_env] for this step (or null = all valid)
  int B, N;
  const h16* wrm;                     // row-major node images
  const h16* wrm16;                   // x3: the 16x16x32 kernel's images (layout.node_rm16) -> csrc/node16.h
  int o_w1, o_w2, o_w3, o_w4;          // element offsets (strides 168/72/136/72)
  const float* wvec;                   // controller side vector (eb2|nb2|nb3|nb4)
  float act_coef, dt, sqrt3;
  const float* act_scale;              // optional device count n_act: coefficient = act_coef / max(n_act, 1)
  const float* gscale;                 // optional device loss scale (fp16): multiplies the coefficient
  h16* dP;            long dp_env;    // (b,i,128) dL/dpooled out
  float4* ego;                         // (B,N) records: dL/ds_t from the node path + gain law + action loss
  float* partial;                      // (gridDim.x, CTRL_NODE_PARTIAL) slabs, accumulated
  const unsigned char* acts; long na_env;   // step t's node activations from the rollout (CtrlArgs.acts)
                                            // or null: the cooperative kernel recomputes them
  int init;                            // 1: the slabs are written, not accumulated (first BPTT step)
  int chunk;                           // agents per workgroup chunk: 32, 64 or 128 (0 = 128); small
                                       // scenes use smaller chunks to spread over more CUs
  // Fused BPTT combine (ctrl.hip fused_combine; cdS != null): G_{t+1} = dS_{t+1} + ego_{t+1} +
  // the edge terms of dEc_{t+1} + the Euler adjoint of G_{t+2} is formed per agent in the prologue
  // (replacing a node_combine launch between reverse steps), used as Gn and written to cGout
  const float4* cdS;   long cds_env;   // dS_{t+1} (B,N) view
  const float4* cego;                  // ego_{t+1} (B,N) contiguous (this kernel then overwrites ego)
  const float4* cdEc;                  // dEc_{t+1} (B,N,K) contiguous
  const int* cptr;     long cptr_env;  // reverse CSR of graph t+1 (per env strides)
  const int* cedges;   long cedges_env;
  const float4* cGn;   long cgn_env;   // G_{t+2} (or null)
  float4* cGout;       long cgo_env;   // G_{t+1} out
  int K;
  int coop;                            // set by the launchers: 32-agent chunks run node_bwd_coop
  unsigned long long* stamps;          // diagnostics (null in production): node_bwd_coop phase clocks,
                                       // [workgroup][wave][16] shader-clock values (scripts/stamps_node.py)
};

// the cooperative 32-agent node backward (node_bwd_coop) runs every 32-agent chunk
inline bool node_bwd_coop_enabled() { return true; }

struct CtrlEdgeBwdArgs {
  const float4* S;     long s_env;     // node records (strides in records)
  int dim;
  const int* idx;      long i_env;
  const uint8_t* argmax; long am_env;  // (b,i,128) winning slot per pooled feature
  const h16* dP;      long dp_env;    // (b,i,128)
  int B, N, K;
  const h16* wpack;   int f_ew1f, f_ew2tn;   // packed fragments (ew2tn followed by ew1ft)
  float4* dEc;         long de_env;    // (b,i,K) records of dL/d(s_i - s_j) out
  float* partial;                      // (gridDim.x, CTRL_EDGE_PARTIAL) slabs, accumulated
  int init;                            // 1: the slabs are written, not accumulated (first BPTT step)
  int qsplit;                          // workgroups per 128-agent chunk (tile-range split; 1, 2, 4, 8, 16)
  const h16* w16;                      // x3, K = 12: 16x16x32 fragments (csrc/ctrl16.h) -> the two-waves-per-SIMD kernel
  unsigned long long* stamps;          // diagnostics or null: [workgroup][wave][16] phase cycles (16x16x32 kernel)
};

struct CsrArgs {
  const int* idx;      // (G, N, K) neighbour indices of G = B*T graphs (N centres)
  int G, N, K;
  int Nn;              // target nodes (agents + obstacle points); 0 = N
  int* ptr;            // (G, Nn+1) incoming-edge offsets
  int* edges;          // (G, N*K) incoming edge ids (i*K + k), self edges excluded
  int* ws;             // (G, Nn) fill counters of the global path (envs whose counters exceed LDS)
};

struct NodeRedArgs {
  const float4* dE;    // (passes, T, B, N, K) per-edge dL/d(s_i - s_j)
  const int* ptr; const int* edges;   // reverse CSR of the B*T graphs
  int B, T, N, K, passes, accumulate;
  float4* out;         // (T+1, B, N)
  int pass_mask;       // bit p: include pass p (0 -> all passes)
  int Nn;              // CSR target nodes per graph (0 = N)
  int dim;
  int shift1;          // pass 1 edges belong to graph t + shift1 (1: h' on recomputed kNN of s_{t+1})
  const int* map1;     // dedup: pass-1 slot e -> evaluation index (only >= E = extras are read)
  const float* gate;   // optional: dE[x] is read only where gate[x] != 0 (the skipped evaluations of
                       // the active-list backward leave their dE records unwritten)
  int t_lo, t_hi;      // output steps t_lo <= t' < t_hi (t_hi = 0: all T+1)
};

struct CombineArgs {
  int dim;                            // records of REC<dim> float4s; strides in records
  const float4* dS;   long ds_env;    // direct grads at step t (B,N) view
  const float4* ego;                  // (B,N) contiguous or null
  const float4* dEc;                  // (B,N,K) controller edge grads at step t or null
  const int* ptr;     long ptr_env;   // reverse CSR of graph t (per env strides)
  const int* edges;   long edges_env;
  const float4* Gn;   long gn_env;    // G_{t+1} (B,N) view, or null (no BPTT / last step)
  float4* Gout;       long go_env;    // G_t (B,N) view
  int B, N, K;
  float dt;
};


struct RolloutStatsArgs {
  unsigned long long* dist;   // (T, B) per-env sum of |p_{t+1} - g| over the N agents (x FX_DIST)
  float* cnt;             // (T, B, 2) dangerous / safe edge counts of step t
  float* safe;            // (T+1, B) safe-agent counts of s_t (or null)
  unsigned long long* act;    // (T, B) per-env action-loss sums (x FX_ACT, or null)
  int T, B, N;
  int reset_T;            // > 0: after reading, zero the Tmax = reset_T rows of dist / cnt / act and the
                          // Tmax + 1 rows of safe (the next rollout's atomics start from zero: no fills)
  float thr;              // DIST_MIN_CHECK
  uint8_t* valid;         // (T, B) out
  float* counts;          // [n_dang, n_safe, n_act] out (this rank)
  float* local;           // [agent-steps, safe agents of s_{t+1}, action-loss sum] out
};

// End of an optimizer step (one thread): step counters or the skipped count, the fp16 dynamic
// loss scale (halved on a non-finite step, doubled after `growth` finite ones), this step's
// statistics row [16] = skipped, [17] = loss scale, and the guard flag reset to 1 for the next step.
struct StepCommitArgs {
  int* ok; int* steps; int mask, ngroups; int* skipped;
  float* gscale; int* good; int growth; float max_scale;   // gscale null: no loss scaling
  float* stats_row;                                        // null: no statistics row
  const float* stats_src;   // optional: stats_row[0:16] copied from here first (graph-replayed backward)
};

struct AdamArgs {
  float* param; const float* grad; float* m; float* v;
  int lo, hi;
  float b1, b2, eps, wd, step_size, bc2_sqrt;
  const int* ok;          // optional device guard flag (0: skip the step)
  const int* step;        // optional device step counter (bias corrections from *step + 1, lr)
  float lr;
};

// several parameter groups' Adam steps in one launch (block offsets filled by the launcher)
constexpr int AM_GROUPS = 4;
struct AdamMultiArgs { AdamArgs g[AM_GROUPS]; int blk0[AM_GROUPS]; int ngroups; };

// several slab reductions in one launch (block offsets filled by the launcher)
constexpr int RM_JOBS = 4;
struct ReduceMultiArgs {
  const float* partial[RM_JOBS]; float* out[RM_JOBS];
  int rows[RM_JOBS], cols[RM_JOBS], accumulate[RM_JOBS], blk0[RM_JOBS];
  int njobs;
};

// flat gradient assembly (+ optional finite check and statistics row)
struct GradAssembleArgs {
  const float* red; const int* ptr; const int* src; int n; float scale; const float* gscale; float* grad;
  int* ok;                                            // null: no check (an all-reduce follows)
  const float* sums; const float* counts; const float* local; float* row;   // row null: no stats
};

}  // namespace mb

extern "C" {
int mb_scan(const mb::ScanArgs* a, hipStream_t st);
int mb_scan_plan(const mb::ScanArgs* a, long* out);
int mb_reduce_multi(const mb::ReduceMultiArgs* a, hipStream_t st);
int mb_adam_multi(const mb::AdamMultiArgs* a, hipStream_t st);
int mb_cell_sort(const mb::CellSortArgs* a, hipStream_t st);
int mb_scenario(const mb::ScenArgs* a, hipStream_t st);
int mb_ctrl_fwd(const mb::CtrlArgs* a, int num_cu, hipStream_t st);
int mb_ctrl_fwd_f16(const mb::CtrlArgs* a, int num_cu, hipStream_t st);
int mb_ctrl_fwd_x3(const mb::CtrlArgs* a, int num_cu, hipStream_t st);
int mb_rollout_small(const mb::RolloutSmallArgs* a, hipStream_t st);
int mb_rollout_small_f16(const mb::RolloutSmallArgs* a, hipStream_t st);
int mb_rollout_small_x3(const mb::RolloutSmallArgs* a, hipStream_t st);
int mb_cbf_fwd(const mb::CbfFwdArgs* a, int num_blocks, hipStream_t st);
int mb_cbf_fwd_f16(const mb::CbfFwdArgs* a, int num_blocks, hipStream_t st);
int mb_cbf_fwd_x3(const mb::CbfFwdArgs* a, int num_blocks, hipStream_t st);
int mb_cbf_hfwd(const mb::CbfFwdArgs* a, int num_blocks, hipStream_t st);
int mb_cbf_hfwd_f16(const mb::CbfFwdArgs* a, int num_blocks, hipStream_t st);
int mb_cbf_hfwd_x3(const mb::CbfFwdArgs* a, int num_blocks, hipStream_t st);
int mb_cbf_bwd(const mb::CbfBwdArgs* a, int num_blocks, hipStream_t st);
int mb_cbf_bwd_f16(const mb::CbfBwdArgs* a, int num_blocks, hipStream_t st);
int mb_cbf_bwd_x3(const mb::CbfBwdArgs* a, int num_blocks, hipStream_t st);
int mb_ctrl_node_bwd(const mb::CtrlNodeBwdArgs* a, int num_blocks, hipStream_t st);
int mb_ctrl_node_bwd_f16(const mb::CtrlNodeBwdArgs* a, int num_blocks, hipStream_t st);
int mb_ctrl_node_bwd_x3(const mb::CtrlNodeBwdArgs* a, int num_blocks, hipStream_t st);
int mb_ctrl_bwd_step(const mb::CtrlNodeBwdArgs* na, const mb::CtrlEdgeBwdArgs* ea, int num_blocks, hipStream_t st);
int mb_ctrl_bwd_step_f16(const mb::CtrlNodeBwdArgs* na, const mb::CtrlEdgeBwdArgs* ea, int num_blocks, hipStream_t st);
int mb_ctrl_bwd_step_x3(const mb::CtrlNodeBwdArgs* na, const mb::CtrlEdgeBwdArgs* ea, int num_blocks, hipStream_t st);
int mb_ctrl_edge_bwd(const mb::CtrlEdgeBwdArgs* a, int num_blocks, hipStream_t st);
int mb_ctrl_edge_bwd_f16(const mb::CtrlEdgeBwdArgs* a, int num_blocks, hipStream_t st);
int mb_ctrl_edge_bwd_x3(const mb::CtrlEdgeBwdArgs* a, int num_blocks, hipStream_t st);
// 16x16x32 backward workgroups per CU of each build (the launch grid; csrc/cbf16.h, csrc/ctrl16.h)
int mb_k16_wg_per_cu(int kernel);
int mb_k16_wg_per_cu_f16(int kernel);
int mb_k16_wg_per_cu_x3(int kernel);
int mb_node_act_bytes();
int mb_node_act_bytes_f16();
int mb_node_act_bytes_x3();
int mb_rev_csr(const mb::CsrArgs* a, hipStream_t st);
int mb_cbf_match(const mb::CbfMatchArgs* a, hipStream_t st);
int mb_cbf_dh(const mb::CbfDhArgs* a, int num_blocks, hipStream_t st);
int mb_cbf_compact(const float* dh, const int* nev, const int* blk_off, int* act, int num_blocks,
                   const int* blk_active, int* nact, const int* src, const int* idx, const int* idx1, unsigned E,
                   void* rec, hipStream_t st);
int mb_node_reduce(const mb::NodeRedArgs* a, hipStream_t st);
int mb_node_combine(const mb::CombineArgs* a, hipStream_t st);
int mb_reduce_rows(const float* partial, int rows, int cols, float* out, int accumulate, hipStream_t st);
int mb_adam(const mb::AdamArgs* a, hipStream_t st);
int mb_rollout_stats(const mb::RolloutStatsArgs* a, hipStream_t st);
int mb_grad_check(const float* g, int n, int* ok, hipStream_t st);
int mb_grad_assemble(const mb::GradAssembleArgs* a, hipStream_t st);
int mb_pack_gather(const float* src, int n, const int* idx16, int m16, unsigned short* out16, int f16,
                   const int* idx32, int m32, float* out32, const mb::StepCommitArgs* commit, hipStream_t st);
int mb_step_commit(const mb::StepCommitArgs* a, hipStream_t st);
int mb_stats_pack(const float* sums, const float* counts, const float* local, float* row, hipStream_t st);
int mb_probe_mfma16(const void* a, const void* b, float* d, hipStream_t st);
int mb_probe_mfma(const void* a, const void* b, float* d, hipStream_t st);
int mb_probe_lane_xor(const unsigned* in, unsigned* out, hipStream_t st);
int mb_probe_tr(const void* img, int rows, int stride, int e0, int m0, void* out, hipStream_t st);
}
