// pybind11 layer: raw-pointer launchers for the gfx950 kernels.
//
// Tensors are validated (device, dtype, contiguity, shape) on the Python side in
// macbf_gnn_amd/ops/native.py and passed here as integer device addresses together with the
// current HIP stream handle of PyTorch, so this module needs no libtorch headers and builds
// in seconds. Every launcher returns the hipError_t of the launch; native.py raises on != 0.
#include <pybind11/pybind11.h>
#include <hip/hip_runtime.h>

#include "args.h"

namespace py = pybind11;
using u64 = unsigned long long;

template <typename T>
static T* P(u64 p) { return reinterpret_cast<T*>(static_cast<uintptr_t>(p)); }
static hipStream_t ST(u64 s) { return reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(s)); }

// loss constants: 7 floats (+ optional device loss-scale pointer)
static mb::LossConsts LC(const py::tuple& lc) {
  mb::LossConsts c{};
  c.eps_dang = lc[0].cast<float>(); c.dt_alpha = lc[1].cast<float>(); c.w_dang = lc[2].cast<float>();
  c.w_safe = lc[3].cast<float>(); c.w_dang_d = lc[4].cast<float>(); c.w_safe_d = lc[5].cast<float>();
  c.scale = lc[6].cast<float>();
  c.gscale = lc.size() > 7 ? P<const float>(lc[7].cast<u64>()) : nullptr;
  return c;
}

static int cell_sort(u64 S, long s_env, int B, int N, float L, u64 perm, int rec, u64 stream) {
  mb::CellSortArgs a{};
  a.rec = rec;
  a.S = P<const float4>(S); a.s_env = s_env; a.B = B; a.N = N; a.L = L; a.perm = P<int>(perm);
  return mb_cell_sort(&a, ST(stream));
}

static int scan(u64 S, long s_env, u64 perm, int B, int N, int K, u64 idx, long i_env, u64 dang, u64 cnt, long c_env,
                u64 safe, long sf_env, float r2_train, float ttc_train, float r2_check, float ttc_check,
                int do_knn, int do_safety, int Nn, int dim, u64 prev_idx, long pi_env, u64 ws, long ws_env,
                int lanes, u64 stamps, u64 stream) {
  mb::ScanArgs a{};
  a.lanes = lanes;
  a.stamps = P<unsigned long long>(stamps);
  a.ws = P<float4>(ws); a.ws_env = ws_env;
  a.prev_idx = P<const int>(prev_idx); a.pi_env = pi_env;
  a.Nn = Nn; a.dim = dim;
  a.S = P<const float4>(S); a.s_env = s_env; a.perm = P<const int>(perm); a.B = B; a.N = N; a.K = K;
  a.idx = P<int>(idx); a.i_env = i_env; a.dang = P<uint8_t>(dang);
  a.cnt = P<float>(cnt); a.c_env = c_env; a.safe = P<float>(safe); a.sf_env = sf_env;
  a.r2_train = r2_train; a.ttc_train = ttc_train; a.r2_check = r2_check; a.ttc_check = ttc_check;
  a.do_knn = do_knn; a.do_safety = do_safety;
  return mb_scan(&a, ST(stream));
}

// the launch plan mb_scan picks for a call of this shape (tests assert the instantiation they hit)
static py::tuple scan_plan(int B, int N, int K, int Nn, int dim, int has_prev, int do_knn, int do_safety, int lanes) {
  mb::ScanArgs a{};
  a.B = B; a.N = N; a.K = K; a.Nn = Nn; a.dim = dim; a.lanes = lanes;
  a.do_knn = do_knn; a.do_safety = do_safety;
  static const int dummy = 0;
  a.prev_idx = has_prev ? &dummy : nullptr;
  long out[9] = {};
  const int rc = mb_scan_plan(&a, out);
  if (rc) throw std::runtime_error("scan_plan: bad arguments");
  return py::make_tuple(out[0], out[1], out[2], out[3], out[4], out[5], out[6], out[7], out[8]);
}

static int scenario(u64 S, long s_env, u64 G, u64 obs, int M, int dim, int B, int N, float L, float r, float spread,
                    u64 seed, int max_rounds, u64 status, u64 ws, long ws_env, u64 stream) {
  mb::ScenArgs a{};
  a.ws = P<unsigned char>(ws); a.ws_env = ws_env;
  a.S = P<float4>(S); a.s_env = s_env; a.G = P<float>(G); a.obs = P<const float>(obs); a.M = M; a.dim = dim;
  a.B = B; a.N = N; a.L = L; a.r = r; a.spread = spread;
  a.seed = seed; a.max_rounds = max_rounds; a.status = P<int>(status);
  return mb_scenario(&a, ST(stream));
}

static int ctrl_fwd(u64 S, long s_env, u64 G, u64 idx, long i_env, int B, int N, int K, u64 wpack, int f_edge,
                    int f_node, u64 wvec, u64 A, long a_env, u64 Sn, long sn_env, u64 dist_sum, long d_env,
                    u64 act_sum, long ac_env, u64 noise, long n_env, float dt, float obs_r, float sqrt3,
                    u64 pooled, long p_env, u64 argmax, long am_env, int dim, int num_cu, int prec, int apw,
                    u64 noise_key, float noise_prob, float noise_scale, int noise_t, u64 stamps, u64 stream) {
  mb::CtrlArgs a{};
  a.stamps = P<unsigned long long>(stamps);
  a.dim = dim;
  a.apw = apw;
  a.S = P<const float4>(S); a.s_env = s_env; a.G = P<const float>(G); a.idx = P<const int>(idx); a.i_env = i_env;
  a.B = B; a.N = N; a.K = K; a.wpack = P<const h16>(wpack); a.f_edge = f_edge; a.f_node = f_node;
  a.wvec = P<const float>(wvec); a.A = P<float>(A); a.a_env = a_env; a.Snext = P<float4>(Sn); a.sn_env = sn_env;
  a.dist_sum = P<unsigned long long>(dist_sum); a.d_env = d_env; a.act_sum = P<unsigned long long>(act_sum);
  a.ac_env = ac_env;
  a.noise = P<const float>(noise); a.n_env = n_env; a.dt = dt; a.obs_r = obs_r; a.sqrt3 = sqrt3;
  a.pooled = P<h16>(pooled); a.p_env = p_env; a.argmax = P<uint8_t>(argmax); a.am_env = am_env;
  a.noise_key = P<const unsigned long long>(noise_key); a.noise_prob = noise_prob; a.noise_scale = noise_scale;
  a.noise_t = noise_t;
  return (prec == 2 ? mb_ctrl_fwd_x3 : prec == 1 ? mb_ctrl_fwd_f16 : mb_ctrl_fwd)(&a, num_cu, ST(stream));
}

static int cbf_fwd(u64 S, long s_env, long s_step, u64 idx, u64 dang, u64 valid, int B, int T, int N, int K,
                   int two, u64 wpack, int f_fwd, u64 wvec, u64 h_out, u64 hn_out, u64 dh_out, u64 counts,
                   u64 partial, py::tuple lc, float obs_r, float dist_thr, float dist_eps, int dim, int num_blocks,
                   int prec, u64 stream) {
  mb::CbfFwdArgs a{};
  a.dim = dim;
  a.S = P<const float4>(S); a.s_env = s_env; a.s_step = s_step; a.idx = P<const int>(idx);
  a.dang = P<const uint8_t>(dang); a.valid = P<const uint8_t>(valid);
  a.B = B; a.T = T; a.N = N; a.K = K; a.two = two;
  a.wpack = P<const h16>(wpack); a.f_fwd = f_fwd; a.wvec = P<const float>(wvec);
  a.h_out = P<float>(h_out); a.hn_out = P<float>(hn_out); a.dh_out = P<float>(dh_out);
  a.counts = P<const float>(counts); a.partial = P<float>(partial);
  a.lc = LC(lc);
  a.obs_r = obs_r; a.dist_thr = dist_thr; a.dist_eps = dist_eps;
  return (prec == 2 ? mb_cbf_fwd_x3 : prec == 1 ? mb_cbf_fwd_f16 : mb_cbf_fwd)(&a, num_blocks, ST(stream));
}

static int cbf_hfwd(u64 S, long s_env, long s_step, u64 idx, u64 idx1, u64 src, u64 nev, int B, int T, int N, int K,
                    u64 wpack, int f_fwd, u64 wrm, u64 wvec, u64 h_out, u64 mask_out, float obs_r, float dist_thr,
                    float dist_eps, int dim, int num_blocks, int prec, unsigned u_begin, unsigned u_end,
                    u64 stream) {
  mb::CbfFwdArgs a{};
  a.dim = dim;
  a.u_begin = u_begin; a.u_end = u_end;
  a.S = P<const float4>(S); a.s_env = s_env; a.s_step = s_step; a.idx = P<const int>(idx);
  a.idx1 = P<const int>(idx1); a.src = P<const int>(src); a.nev = P<const int>(nev);
  a.B = B; a.T = T; a.N = N; a.K = K; a.two = 1;
  a.wpack = P<const h16>(wpack); a.f_fwd = f_fwd; a.wrm = P<const h16>(wrm); a.wvec = P<const float>(wvec);
  a.h_out = P<float>(h_out); a.mask_out = P<uint8_t>(mask_out);
  a.obs_r = obs_r; a.dist_thr = dist_thr; a.dist_eps = dist_eps;
  return (prec == 2 ? mb_cbf_hfwd_x3 : prec == 1 ? mb_cbf_hfwd_f16 : mb_cbf_hfwd)(&a, num_blocks, ST(stream));
}

static int cbf_bwd(u64 S, long s_env, long s_step, u64 idx, int B, int T, int N, int K, int passes, u64 dh,
                   u64 wpack, int f_bwd, u64 wrm, u64 wvec, u64 dE, u64 partial, float obs_r, float dist_thr,
                   float dist_eps, int fused, u64 dang, u64 valid, u64 counts, py::tuple lc, u64 idx1,
                   int dim, int num_blocks, int prec, u64 src, u64 nev, u64 act, u64 nact, u64 rec, u64 wrm16, u64 w16,
                   u64 dbg, u64 stamps, u64 stream) {
  mb::CbfBwdArgs a{};
  a.stamps = P<unsigned long long>(stamps);
  a.rec = P<const int4>(rec); a.wrm16 = P<const h16>(wrm16); a.w16 = P<const h16>(w16);
  a.dbg = P<float>(dbg);
  a.dim = dim;
  a.src = P<const int>(src); a.nev = P<const int>(nev); a.act = P<const int>(act); a.nact = P<const int>(nact);
  a.idx1 = P<const int>(idx1);
  a.fused = fused; a.dang = P<const uint8_t>(dang); a.valid = P<const uint8_t>(valid);
  a.counts = P<const float>(counts);
  a.lc = LC(lc);
  a.S = P<const float4>(S); a.s_env = s_env; a.s_step = s_step; a.idx = P<const int>(idx);
  a.B = B; a.T = T; a.N = N; a.K = K; a.passes = passes; a.dh = P<const float>(dh);
  a.wpack = P<const h16>(wpack); a.f_bwd = f_bwd; a.wrm = P<const h16>(wrm); a.wvec = P<const float>(wvec);
  a.dE = P<float4>(dE); a.partial = P<float>(partial);
  a.obs_r = obs_r; a.dist_thr = dist_thr; a.dist_eps = dist_eps;
  return (prec == 2 ? mb_cbf_bwd_x3 : prec == 1 ? mb_cbf_bwd_f16 : mb_cbf_bwd)(&a, num_blocks, ST(stream));
}

static int rev_csr(u64 idx, int G, int N, int K, u64 ptr, u64 edges, int Nn, u64 ws, u64 stream) {
  mb::CsrArgs a{};
  a.Nn = Nn;
  a.ws = P<int>(ws);
  a.idx = P<const int>(idx); a.G = G; a.N = N; a.K = K; a.ptr = P<int>(ptr); a.edges = P<int>(edges);
  return mb_rev_csr(&a, ST(stream));
}

static int node_reduce(u64 dE, u64 ptr, u64 edges, int B, int T, int N, int K, int passes, int accumulate, u64 out,
                       int pass_mask, int shift1, int Nn, int dim, u64 map1, u64 gate, int t_lo, int t_hi,
                       u64 stream) {
  mb::NodeRedArgs a{};
  a.t_lo = t_lo; a.t_hi = t_hi;
  a.map1 = P<const int>(map1); a.gate = P<const float>(gate);
  a.pass_mask = pass_mask; a.shift1 = shift1; a.Nn = Nn; a.dim = dim;
  a.dE = P<const float4>(dE); a.ptr = P<const int>(ptr); a.edges = P<const int>(edges);
  a.B = B; a.T = T; a.N = N; a.K = K; a.passes = passes; a.accumulate = accumulate; a.out = P<float4>(out);
  return mb_node_reduce(&a, ST(stream));
}

static int cbf_match(u64 idx, int T, int B, int N, int K, int mode, int phase, u64 cnt, u64 off, u64 map1, u64 src,
                     u64 bsum, u64 nev, u64 stream) {
  mb::CbfMatchArgs a{};
  a.idx = P<const int>(idx); a.T = T; a.B = B; a.N = N; a.K = K; a.mode = mode; a.phase = phase;
  a.cnt = P<int>(cnt); a.off = P<const int>(off); a.map1 = P<int>(map1); a.src = P<int>(src);
  a.bsum = P<int>(bsum); a.nev = P<int>(nev);
  return mb_cbf_match(&a, ST(stream));
}

static int cbf_dh(u64 h, u64 hmask, u64 map1, u64 src, u64 nev, u64 dang, u64 valid, int B, int T, int N, int K,
                  u64 counts, py::tuple lc, u64 dh, u64 partial, u64 blk_active, int num_blocks, u64 stream) {
  mb::CbfDhArgs a{};
  a.blk_active = P<int>(blk_active);
  a.h = P<const float>(h); a.hmask = P<const uint8_t>(hmask); a.map1 = P<const int>(map1);
  a.src = P<const int>(src); a.nev = P<const int>(nev); a.dang = P<const uint8_t>(dang);
  a.valid = P<const uint8_t>(valid); a.B = B; a.T = T; a.N = N; a.K = K; a.counts = P<const float>(counts);
  a.lc = LC(lc);
  a.dh = P<float>(dh); a.partial = P<float>(partial);
  return mb_cbf_dh(&a, num_blocks, ST(stream));
}

static int cbf_compact(u64 dh, u64 nev, u64 blk_off, u64 act, int num_blocks, u64 blk_active, u64 nact,
                       u64 src, u64 idx, u64 idx1, unsigned E, u64 rec, u64 stream) {
  return mb_cbf_compact(P<const float>(dh), P<const int>(nev), P<const int>(blk_off), P<int>(act), num_blocks,
                        P<const int>(blk_active), P<int>(nact), P<const int>(src), P<const int>(idx),
                        P<const int>(idx1), E, P<void>(rec), ST(stream));
}

static int node_combine(u64 dS, long ds_env, u64 ego, u64 dEc, u64 ptr, long ptr_env, u64 edges, long edges_env,
                        u64 Gn, long gn_env, u64 Gout, long go_env, int B, int N, int K, float dt, int dim,
                        u64 stream) {
  mb::CombineArgs a{};
  a.dim = dim;
  a.dS = P<const float4>(dS); a.ds_env = ds_env; a.ego = P<const float4>(ego); a.dEc = P<const float4>(dEc);
  a.ptr = P<const int>(ptr); a.ptr_env = ptr_env; a.edges = P<const int>(edges); a.edges_env = edges_env;
  a.Gn = P<const float4>(Gn); a.gn_env = gn_env; a.Gout = P<float4>(Gout); a.go_env = go_env;
  a.B = B; a.N = N; a.K = K; a.dt = dt;
  return mb_node_combine(&a, ST(stream));
}

static int reduce_rows(u64 partial, int rows, int cols, u64 out, int accumulate, u64 stream) {
  return mb_reduce_rows(P<const float>(partial), rows, cols, P<float>(out), accumulate, ST(stream));
}

static mb::StepCommitArgs commit_args(u64 ok, u64 steps, int mask, int ngroups, u64 skipped, u64 gscale, u64 good,
                                      int growth, float max_scale, u64 stats_row, u64 stats_src = 0) {
  mb::StepCommitArgs a{};
  a.ok = P<int>(ok); a.steps = P<int>(steps); a.mask = mask; a.ngroups = ngroups; a.skipped = P<int>(skipped);
  a.gscale = P<float>(gscale); a.good = P<int>(good); a.growth = growth; a.max_scale = max_scale;
  a.stats_row = P<float>(stats_row);
  a.stats_src = P<const float>(stats_src);
  return a;
}

// commit: None, or the step_commit arguments (ok, steps, mask, ngroups, skipped, gscale, good, growth,
// max_scale, stats_row[, stats_src]) -- the optimizer step's commit runs inside the gather launch
static int pack_gather(u64 src, int n, u64 idx16, int m16, u64 out16, int f16, u64 idx32, int m32, u64 out32,
                       py::object commit, u64 stream) {
  mb::StepCommitArgs c{};
  const bool has = !commit.is_none();
  if (has) {
    const py::tuple t = commit.cast<py::tuple>();
    c = commit_args(t[0].cast<u64>(), t[1].cast<u64>(), t[2].cast<int>(), t[3].cast<int>(), t[4].cast<u64>(),
                    t[5].cast<u64>(), t[6].cast<u64>(), t[7].cast<int>(), t[8].cast<float>(), t[9].cast<u64>(),
                    t.size() > 10 ? t[10].cast<u64>() : 0);
  }
  return mb_pack_gather(P<const float>(src), n, P<const int>(idx16), m16, P<unsigned short>(out16), f16,
                        P<const int>(idx32), m32, P<float>(out32), has ? &c : nullptr, ST(stream));
}

static int grad_assemble(u64 red, u64 ptr, u64 src, int n, float scale, u64 gscale, u64 grad, u64 ok, u64 sums,
                         u64 counts, u64 local, u64 row, u64 stream) {
  mb::GradAssembleArgs a{};
  a.red = P<const float>(red); a.ptr = P<const int>(ptr); a.src = P<const int>(src); a.n = n; a.scale = scale;
  a.gscale = P<const float>(gscale); a.grad = P<float>(grad); a.ok = P<int>(ok);
  a.sums = P<const float>(sums); a.counts = P<const float>(counts); a.local = P<const float>(local); a.row = P<float>(row);
  return mb_grad_assemble(&a, ST(stream));
}

// jobs: [(partial, rows, cols, out, accumulate)] (at most mb::RM_JOBS), one launch
static int reduce_multi(py::list jobs, u64 stream) {
  mb::ReduceMultiArgs a{};
  a.njobs = (int)py::len(jobs);
  if (a.njobs < 1 || a.njobs > mb::RM_JOBS) return -1;
  for (int j = 0; j < a.njobs; ++j) {
    const py::tuple t = jobs[j].cast<py::tuple>();
    a.partial[j] = P<const float>(t[0].cast<u64>()); a.rows[j] = t[1].cast<int>(); a.cols[j] = t[2].cast<int>();
    a.out[j] = P<float>(t[3].cast<u64>()); a.accumulate[j] = t[4].cast<int>();
  }
  return mb_reduce_multi(&a, ST(stream));
}

// groups: [(lo, hi, step_ptr)] (at most mb::AM_GROUPS); the rest as adam()
static int adam_multi(u64 param, u64 grad, u64 m, u64 v, py::list groups, float b1, float b2, float eps, float wd,
                      u64 ok, float lr, u64 stream) {
  mb::AdamMultiArgs a{};
  a.ngroups = (int)py::len(groups);
  if (a.ngroups < 1 || a.ngroups > mb::AM_GROUPS) return -1;
  for (int g = 0; g < a.ngroups; ++g) {
    const py::tuple t = groups[g].cast<py::tuple>();
    mb::AdamArgs& x = a.g[g];
    x.param = P<float>(param); x.grad = P<const float>(grad); x.m = P<float>(m); x.v = P<float>(v);
    x.lo = t[0].cast<int>(); x.hi = t[1].cast<int>(); x.step = P<const int>(t[2].cast<u64>());
    x.b1 = b1; x.b2 = b2; x.eps = eps; x.wd = wd; x.ok = P<const int>(ok); x.lr = lr;
    if (!x.step) return -2;          // device step counters only (bias corrections on the device)
  }
  return mb_adam_multi(&a, ST(stream));
}

static int grad_check(u64 g, int n, u64 ok, u64 stream) { return mb_grad_check(P<const float>(g), n, P<int>(ok), ST(stream)); }

static int step_commit(u64 ok, u64 steps, int mask, int ngroups, u64 skipped, u64 gscale, u64 good, int growth,
                       float max_scale, u64 stats_row, u64 stats_src, u64 stream) {
  const mb::StepCommitArgs a = commit_args(ok, steps, mask, ngroups, skipped, gscale, good, growth, max_scale, stats_row,
                                           stats_src);
  return mb_step_commit(&a, ST(stream));
}

static int stats_pack(u64 sums, u64 counts, u64 local, u64 row, u64 stream) {
  return mb_stats_pack(P<const float>(sums), P<const float>(counts), P<const float>(local), P<float>(row), ST(stream));
}

static int rollout_stats(u64 dist, u64 cnt, u64 safe, u64 act, int T, int B, int N, float thr, u64 valid,
                         u64 counts, u64 local, int reset_T, u64 stream) {
  mb::RolloutStatsArgs a{};
  a.reset_T = reset_T;
  a.dist = P<unsigned long long>(dist); a.cnt = P<float>(cnt); a.safe = P<float>(safe);
  a.act = P<unsigned long long>(act); a.T = T; a.B = B; a.N = N; a.thr = thr; a.valid = P<uint8_t>(valid);
  a.counts = P<float>(counts); a.local = P<float>(local);
  return mb_rollout_stats(&a, ST(stream));
}

static int adam(u64 param, u64 grad, u64 m, u64 v, int lo, int hi, float b1, float b2, float eps, float wd,
                float step_size, float bc2_sqrt, u64 ok, u64 step, float lr, u64 stream) {
  mb::AdamArgs a{};
  a.ok = P<const int>(ok); a.step = P<const int>(step); a.lr = lr;
  a.param = P<float>(param); a.grad = P<const float>(grad); a.m = P<float>(m); a.v = P<float>(v);
  a.lo = lo; a.hi = hi; a.b1 = b1; a.b2 = b2; a.eps = eps; a.wd = wd; a.step_size = step_size; a.bc2_sqrt = bc2_sqrt;
  return mb_adam(&a, ST(stream));
}

#define NODE_BWD_PARAMS                                                                                     \
  u64 pooled, long p_env, u64 S, long s_env, u64 G, u64 A, long a_env, u64 Gn, long gn_env, u64 valid, long v_env, \
      int B, int N, u64 wrm, int o1, int o2, int o3, int o4, u64 wvec, float act_coef, u64 act_scale, float dt,    \
      float sqrt3, u64 dP, long dp_env, u64 ego, u64 partial, int dim, int num_blocks, int prec, int init,          \
      int chunk, u64 gscale, py::tuple cmb, u64 stamps
#define NODE_BWD_ARGS                                                                                         \
  pooled, p_env, S, s_env, G, A, a_env, Gn, gn_env, valid, v_env, B, N, wrm, o1, o2, o3, o4, wvec, act_coef,    \
      act_scale, dt, sqrt3, dP, dp_env, ego, partial, dim, num_blocks, prec, init, chunk, gscale, cmb, stamps

static mb::CtrlNodeBwdArgs node_bwd_args(NODE_BWD_PARAMS) {
  (void)num_blocks; (void)prec;
  mb::CtrlNodeBwdArgs a{};
  a.gscale = P<const float>(gscale);
  a.stamps = P<unsigned long long>(stamps);
  if (cmb.size() == 13) {     // fused BPTT combine: (dS, ds_env, ego, dEc, ptr, ptr_env, edges, edges_env, Gn, gn_env,
                              //                     Gout, go_env, K)
    a.cdS = P<const float4>(cmb[0].cast<u64>()); a.cds_env = cmb[1].cast<long>();
    a.cego = P<const float4>(cmb[2].cast<u64>()); a.cdEc = P<const float4>(cmb[3].cast<u64>());
    a.cptr = P<const int>(cmb[4].cast<u64>()); a.cptr_env = cmb[5].cast<long>();
    a.cedges = P<const int>(cmb[6].cast<u64>()); a.cedges_env = cmb[7].cast<long>();
    a.cGn = P<const float4>(cmb[8].cast<u64>()); a.cgn_env = cmb[9].cast<long>();
    a.cGout = P<float4>(cmb[10].cast<u64>()); a.cgo_env = cmb[11].cast<long>();
    a.K = cmb[12].cast<int>();
  }
  a.init = init;
  a.chunk = chunk;
  a.dim = dim;
  a.pooled = P<const h16>(pooled); a.p_env = p_env; a.S = P<const float4>(S); a.s_env = s_env;
  a.G = P<const float>(G); a.A = P<const float>(A); a.a_env = a_env; a.Gn = P<const float4>(Gn); a.gn_env = gn_env;
  a.valid = P<const uint8_t>(valid); a.v_env = v_env; a.B = B; a.N = N; a.wrm = P<const h16>(wrm);
  a.o_w1 = o1; a.o_w2 = o2; a.o_w3 = o3; a.o_w4 = o4; a.wvec = P<const float>(wvec);
  a.act_coef = act_coef; a.act_scale = P<const float>(act_scale); a.dt = dt; a.sqrt3 = sqrt3; a.dP = P<h16>(dP); a.dp_env = dp_env;
  a.ego = P<float4>(ego); a.partial = P<float>(partial);
  return a;
}

static int ctrl_node_bwd(NODE_BWD_PARAMS, u64 wrm16, u64 stream) {
  mb::CtrlNodeBwdArgs a = node_bwd_args(NODE_BWD_ARGS);
  a.wrm16 = P<const h16>(wrm16);      // x3, 128-agent chunks: the 16x16x32 kernel (csrc/node16.h)
  return (prec == 2 ? mb_ctrl_node_bwd_x3 : prec == 1 ? mb_ctrl_node_bwd_f16 : mb_ctrl_node_bwd)(&a, num_blocks, ST(stream));
}

#define EDGE_BWD_PARAMS                                                                                     \
  u64 S, long s_env, u64 idx, long i_env, u64 argmax, long am_env, u64 dP, long dp_env, int B, int N, int K,  \
      u64 wpack, int f_ew1f, int f_ew2tn, u64 dEc, long de_env, u64 partial, int dim, int num_blocks, int prec, \
      int qsplit, int init
#define EDGE_BWD_ARGS \
  S, s_env, idx, i_env, argmax, am_env, dP, dp_env, B, N, K, wpack, f_ew1f, f_ew2tn, dEc, de_env, partial, dim, num_blocks, prec, qsplit, init

static mb::CtrlEdgeBwdArgs edge_bwd_args(EDGE_BWD_PARAMS) {
  (void)num_blocks; (void)prec;
  mb::CtrlEdgeBwdArgs a{};
  a.init = init;
  a.dim = dim;
  a.qsplit = qsplit;
  a.S = P<const float4>(S); a.s_env = s_env; a.idx = P<const int>(idx); a.i_env = i_env;
  a.argmax = P<const uint8_t>(argmax); a.am_env = am_env; a.dP = P<const h16>(dP); a.dp_env = dp_env;
  a.B = B; a.N = N; a.K = K; a.wpack = P<const h16>(wpack); a.f_ew1f = f_ew1f; a.f_ew2tn = f_ew2tn;
  a.dEc = P<float4>(dEc); a.de_env = de_env; a.partial = P<float>(partial);
  return a;
}

static int ctrl_edge_bwd(EDGE_BWD_PARAMS, u64 w16, u64 stamps, u64 stream) {
  mb::CtrlEdgeBwdArgs a = edge_bwd_args(EDGE_BWD_ARGS);
  a.w16 = P<const h16>(w16);
  a.stamps = P<unsigned long long>(stamps);
  return (prec == 2 ? mb_ctrl_edge_bwd_x3 : prec == 1 ? mb_ctrl_edge_bwd_f16 : mb_ctrl_edge_bwd)(&a, num_blocks, ST(stream));
}

// One fused BPTT step (ctrl.hip ctrl_bwd_step_kernel): `node` and `edge` are the argument tuples
// of ctrl_node_bwd / ctrl_edge_bwd without the stream; one launch of num_blocks workgroups.
static int ctrl_bwd_step(py::tuple node, py::tuple edge, int num_blocks, int prec, u64 stream) {
  if (node.size() != 35 || edge.size() != 22) throw std::invalid_argument("ctrl_bwd_step: bad argument tuples");
  auto n = [&](int i) { return node[i]; };
  const mb::CtrlNodeBwdArgs na = node_bwd_args(
      n(0).cast<u64>(), n(1).cast<long>(), n(2).cast<u64>(), n(3).cast<long>(), n(4).cast<u64>(), n(5).cast<u64>(),
      n(6).cast<long>(), n(7).cast<u64>(), n(8).cast<long>(), n(9).cast<u64>(), n(10).cast<long>(), n(11).cast<int>(),
      n(12).cast<int>(), n(13).cast<u64>(), n(14).cast<int>(), n(15).cast<int>(), n(16).cast<int>(), n(17).cast<int>(),
      n(18).cast<u64>(), n(19).cast<float>(), n(20).cast<u64>(), n(21).cast<float>(), n(22).cast<float>(),
      n(23).cast<u64>(), n(24).cast<long>(), n(25).cast<u64>(), n(26).cast<u64>(), n(27).cast<int>(), n(28).cast<int>(),
      n(29).cast<int>(), n(30).cast<int>(), n(31).cast<int>(), n(32).cast<u64>(), n(33).cast<py::tuple>(),
      n(34).cast<u64>());
  auto e = [&](int i) { return edge[i]; };
  const mb::CtrlEdgeBwdArgs ea = edge_bwd_args(
      e(0).cast<u64>(), e(1).cast<long>(), e(2).cast<u64>(), e(3).cast<long>(), e(4).cast<u64>(), e(5).cast<long>(),
      e(6).cast<u64>(), e(7).cast<long>(), e(8).cast<int>(), e(9).cast<int>(), e(10).cast<int>(), e(11).cast<u64>(),
      e(12).cast<int>(), e(13).cast<int>(), e(14).cast<u64>(), e(15).cast<long>(), e(16).cast<u64>(), e(17).cast<int>(),
      e(18).cast<int>(), e(19).cast<int>(), e(20).cast<int>(), e(21).cast<int>());
  return (prec == 2 ? mb_ctrl_bwd_step_x3 : prec == 1 ? mb_ctrl_bwd_step_f16 : mb_ctrl_bwd_step)(&na, &ea, num_blocks,
                                                                                                 ST(stream));
}

static py::dict device_info(int dev) {
  hipDeviceProp_t p;
  py::dict d;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return d;
  d["name"] = std::string(p.name);
  d["gcn_arch"] = std::string(p.gcnArchName);
  d["cu"] = p.multiProcessorCount;
  d["lds_per_block"] = (long)p.sharedMemPerBlock;
  d["warp"] = p.warpSize;
  return d;
}

static std::string err_str(int e) { return hipGetErrorString((hipError_t)e); }

// workgroups per CU of the 16x16x32 backward kernels of build `prec` (kernel 0 CBF, 1 edge, 2 node)
static int node_act_bytes(int prec) {
  return (prec == 2 ? mb_node_act_bytes_x3 : prec == 1 ? mb_node_act_bytes_f16 : mb_node_act_bytes)();
}

static int k16_wg_per_cu(int prec, int kernel) {
  return (prec == 2 ? mb_k16_wg_per_cu_x3 : prec == 1 ? mb_k16_wg_per_cu_f16 : mb_k16_wg_per_cu)(kernel);
}

void register_runtime(py::module& m);   // runtime.cpp: native rollout driver

PYBIND11_MODULE(_C, m) {
  m.doc() = "macbf_gnn_amd native gfx950 kernels";
  register_runtime(m);
  m.def("scan", &scan);
  m.def("scan_plan", &scan_plan);
  m.def("cell_sort", &cell_sort);
  m.def("scenario", &scenario);
  m.def("ctrl_fwd", &ctrl_fwd);
  m.def("cbf_fwd", &cbf_fwd);
  m.def("cbf_bwd", &cbf_bwd);
  m.def("cbf_hfwd", &cbf_hfwd);
  m.def("ctrl_node_bwd", &ctrl_node_bwd);
  m.def("ctrl_edge_bwd", &ctrl_edge_bwd);
  m.def("rev_csr", &rev_csr);
  m.def("node_reduce", &node_reduce);
  m.def("node_combine", &node_combine);
  m.def("cbf_match", &cbf_match);
  m.def("cbf_dh", &cbf_dh);
  m.def("cbf_compact", &cbf_compact);
  m.def("reduce_rows", &reduce_rows);
  m.def("adam", &adam);
  m.def("rollout_stats", &rollout_stats);
  m.def("grad_check", &grad_check);
  m.def("grad_assemble", &grad_assemble);
  m.def("reduce_multi", &reduce_multi);
  m.def("adam_multi", &adam_multi);
  m.def("pack_gather", &pack_gather);
  m.def("step_commit", &step_commit);
  m.def("stats_pack", &stats_pack);
  m.def("ctrl_bwd_step", &ctrl_bwd_step);
  m.def("device_info", &device_info);
  m.def("err_str", &err_str);
  m.def("k16_wg_per_cu", &k16_wg_per_cu);
  m.def("node_act_bytes", &node_act_bytes);
  m.attr("ARCH") = "gfx950";
}
