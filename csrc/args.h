// Kernel argument structs shared by the HIP sources and the pybind11 layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;

namespace mb {

struct ScanArgs {
  const float4* S;  long s_env;      // agent (b,i) state at S[b*s_env + i]
  int B, N, K;
  int* idx;         long i_env;      // (b,i,k) at idx[b*i_env + i*K + k]
  uint8_t* dang;                     // same indexing as idx (may be null)
  float* cnt;       long c_env;      // cnt[b*c_env + {0: dangerous edges, 1: safe edges}]
  float* safe;      long sf_env;     // safe[b*sf_env] += #agents with no dangerous pair
  float r2_train, ttc_train, r2_check, ttc_check;
  int do_knn, do_safety;
};

struct ScenArgs {
  float4* S;      // (B, N) states out (x, y, 0, 0)
  float2* G;      // (B, N) goals out
  int B, N;
  float L, r, spread;
  unsigned long long seed;
  int max_rounds;
  int* status;    // per env: rounds used for goals (or -1 if max_rounds hit)
};

struct CtrlArgs {
  const float4* S;  long s_env;       // states at step t: (b,i) -> S[b*s_env + i]
  const float2* G;                    // goals (b,i) -> G[b*N + i]
  const int* idx;   long i_env;       // (b,i,k) -> idx[b*i_env + i*K + k]
  int B, N, K;
  const bf16* wpack;                  // packed ctrl fragments
  int f_edge;                         // fragment offset of ew1f (ew2 follows)
  int f_node;                         // fragment offset of nw1f (nw2, nw3, nw4 follow)
  const float* wvec;                  // eb2|nb2|nb3|nb4 (CTRL_VEC floats)
  float2* A;        long a_env;       // actions out (may be null)
  float4* Snext;    long sn_env;      // next states out (may be null)
  float* dist_sum;  long d_env;       // per-env sum of |p' - g| (may be null)
  float* act_sum;   long ac_env;      // per-env sum of |‖a‖² - ‖a_ref‖²| (may be null)
  const float2* noise; long n_env;    // additive action noise (may be null)
  float dt, obs_r, sqrt3;
};

struct LossConsts {
  float eps_dang, dt_alpha, w_dang, w_safe, w_dang_d, w_safe_d, scale;
};

struct CbfFwdArgs {
  const float4* S;  long s_env, s_step;   // state of (b,t,i): S[b*s_env + t*s_step + i]
  const int* idx;                          // (B,T,N,K) contiguous
  const uint8_t* dang;                     // (B,T,N,K) or null (all safe)
  const uint8_t* valid;                    // (B,T) or null (all valid)
  int B, T, N, K;
  int two;                                 // also evaluate h' on s_{t+1}
  const bf16* wpack; int f_fwd;            // fragment offset of w1f (w2, w3 follow)
  const float* wvec;
  float* h_out;                            // (E) or null
  float* hn_out;                           // (E) or null
  float* dh_out;                           // (2,E) or null: [dL/dh ; dL/dh']
  const float* counts;                     // device [n_dang, n_safe] (global) for dh
  float* partial;                          // (gridDim.x, 10) or null
  LossConsts lc;
  float obs_r, dist_thr, dist_eps;
};

}  // namespace mb

extern "C" {
int mb_scan(const mb::ScanArgs* a, hipStream_t st);
int mb_scenario(const mb::ScenArgs* a, hipStream_t st);
int mb_ctrl_fwd(const mb::CtrlArgs* a, int num_cu, hipStream_t st);
int mb_cbf_fwd(const mb::CbfFwdArgs* a, int num_blocks, hipStream_t st);
int mb_probe_mfma(const void* a, const void* b, float* d, hipStream_t st);
int mb_probe_tr(const void* img, int rows, int stride, int e0, int m0, void* out, hipStream_t st);
}
