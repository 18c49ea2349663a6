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

static int scan(u64 S, long s_env, int B, int N, int K, u64 idx, long i_env, u64 dang, u64 cnt, long c_env,
                u64 safe, long sf_env, float r2_train, float ttc_train, float r2_check, float ttc_check,
                int do_knn, int do_safety, u64 stream) {
  mb::ScanArgs a{};
  a.S = P<const float4>(S); a.s_env = s_env; a.B = B; a.N = N; a.K = K;
  a.idx = P<int>(idx); a.i_env = i_env; a.dang = P<uint8_t>(dang);
  a.cnt = P<float>(cnt); a.c_env = c_env; a.safe = P<float>(safe); a.sf_env = sf_env;
  a.r2_train = r2_train; a.ttc_train = ttc_train; a.r2_check = r2_check; a.ttc_check = ttc_check;
  a.do_knn = do_knn; a.do_safety = do_safety;
  return mb_scan(&a, ST(stream));
}

static int scenario(u64 S, u64 G, int B, int N, float L, float r, float spread, u64 seed, int max_rounds,
                    u64 status, u64 stream) {
  mb::ScenArgs a{};
  a.S = P<float4>(S); a.G = P<float2>(G); a.B = B; a.N = N; a.L = L; a.r = r; a.spread = spread;
  a.seed = seed; a.max_rounds = max_rounds; a.status = P<int>(status);
  return mb_scenario(&a, ST(stream));
}

static int ctrl_fwd(u64 S, long s_env, u64 G, u64 idx, long i_env, int B, int N, int K, u64 wpack, int f_edge,
                    int f_node, u64 wvec, u64 A, long a_env, u64 Sn, long sn_env, u64 dist_sum, long d_env,
                    u64 act_sum, long ac_env, u64 noise, long n_env, float dt, float obs_r, float sqrt3,
                    int num_cu, u64 stream) {
  mb::CtrlArgs a{};
  a.S = P<const float4>(S); a.s_env = s_env; a.G = P<const float2>(G); a.idx = P<const int>(idx); a.i_env = i_env;
  a.B = B; a.N = N; a.K = K; a.wpack = P<const bf16>(wpack); a.f_edge = f_edge; a.f_node = f_node;
  a.wvec = P<const float>(wvec); a.A = P<float2>(A); a.a_env = a_env; a.Snext = P<float4>(Sn); a.sn_env = sn_env;
  a.dist_sum = P<float>(dist_sum); a.d_env = d_env; a.act_sum = P<float>(act_sum); a.ac_env = ac_env;
  a.noise = P<const float2>(noise); a.n_env = n_env; a.dt = dt; a.obs_r = obs_r; a.sqrt3 = sqrt3;
  return mb_ctrl_fwd(&a, num_cu, ST(stream));
}

static int cbf_fwd(u64 S, long s_env, long s_step, u64 idx, u64 dang, u64 valid, int B, int T, int N, int K,
                   int two, u64 wpack, int f_fwd, u64 wvec, u64 h_out, u64 hn_out, u64 dh_out, u64 counts,
                   u64 partial, py::tuple lc, float obs_r, float dist_thr, float dist_eps, int num_blocks,
                   u64 stream) {
  mb::CbfFwdArgs a{};
  a.S = P<const float4>(S); a.s_env = s_env; a.s_step = s_step; a.idx = P<const int>(idx);
  a.dang = P<const uint8_t>(dang); a.valid = P<const uint8_t>(valid);
  a.B = B; a.T = T; a.N = N; a.K = K; a.two = two;
  a.wpack = P<const bf16>(wpack); a.f_fwd = f_fwd; a.wvec = P<const float>(wvec);
  a.h_out = P<float>(h_out); a.hn_out = P<float>(hn_out); a.dh_out = P<float>(dh_out);
  a.counts = P<const float>(counts); a.partial = P<float>(partial);
  a.lc.eps_dang = lc[0].cast<float>(); a.lc.dt_alpha = lc[1].cast<float>(); a.lc.w_dang = lc[2].cast<float>();
  a.lc.w_safe = lc[3].cast<float>(); a.lc.w_dang_d = lc[4].cast<float>(); a.lc.w_safe_d = lc[5].cast<float>();
  a.lc.scale = lc[6].cast<float>();
  a.obs_r = obs_r; a.dist_thr = dist_thr; a.dist_eps = dist_eps;
  return mb_cbf_fwd(&a, num_blocks, ST(stream));
}

static int probe_mfma(u64 a, u64 b, u64 d, u64 stream) {
  return mb_probe_mfma(P<const void>(a), P<const void>(b), P<float>(d), ST(stream));
}
static int probe_tr(u64 img, int rows, int stride, int e0, int m0, u64 out, u64 stream) {
  return mb_probe_tr(P<const void>(img), rows, stride, e0, m0, P<void>(out), ST(stream));
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

PYBIND11_MODULE(_C, m) {
  m.doc() = "macbf_gnn_amd native gfx950 kernels";
  m.def("scan", &scan);
  m.def("scenario", &scenario);
  m.def("ctrl_fwd", &ctrl_fwd);
  m.def("cbf_fwd", &cbf_fwd);
  m.def("probe_mfma", &probe_mfma);
  m.def("probe_tr", &probe_tr);
  m.def("device_info", &device_info);
  m.def("err_str", &err_str);
  m.attr("ARCH") = "gfx950";
}
