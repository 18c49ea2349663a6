// Native rollout driver: the per-step launch loop of the training rollout in C++.
//
// Reference: the inner loop of train.py:58-81 (controller step, Euler step, early break when
// mean |p - g| < DIST_MIN_CHECK) with the kNN/TTC scan of every step. The Python loop paid
// ~10 wrapper calls per step on the host while the GPU finishes a step in ~0.13 ms at
// 1024 agents x 64 envs, so the host fell behind and the GPU idled between steps. Here the
// argument structs of every step are pointer offsets of persistent buffers validated once on
// the Python side (engine/hip_engine.py), and the loop issues per step:
//   [side stream] CBF h of the previous step's main slots (overlapped with this step)
//   cell_sort (every resort_every steps) + scan, ctrl_fwd
//   [copy stream] per-env goal-distance sums -> pinned host memory
// and checks the early-stop criterion one step late (never stalls the queue on the step just
// issued). Per-env done masks are applied on the device afterwards (rollout_stats).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <tuple>
#include <vector>

#include "args.h"

namespace py = pybind11;
using u64 = unsigned long long;

namespace {

template <typename T>
T* P(u64 p) { return reinterpret_cast<T*>(static_cast<uintptr_t>(p)); }
hipStream_t ST(u64 s) { return reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(s)); }

void chk(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
void chk(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string(what) + " launch failed: " + std::to_string(rc));
}

class RolloutDriver {
 public:
  explicit RolloutDriver(py::dict c) {
    auto I = [&](const char* k) { return c[k].cast<long>(); };
    auto F = [&](const char* k) { return c[k].cast<float>(); };
    auto U = [&](const char* k) { return c[k].cast<u64>(); };
    B_ = (int)I("B"); N_ = (int)I("N"); Nn_ = (int)I("Nn"); K_ = (int)I("K"); D_ = (int)I("D");
    W_ = D_ == 2 ? 4 : 8;
    Tmax_ = (int)I("Tmax"); num_cu_ = (int)I("num_cu"); prec_ = (int)I("prec"); prow_ = prec_ == 2 ? 256 : 128;
    resort_ = (int)I("resort_every"); safety_ = (int)I("compute_safety"); overlap_ = (int)I("overlap_hfwd");
    hfwd_blocks_ = (int)I("hfwd_blocks");
    L_ = F("L");
    S_ = U("S"); G_ = U("G"); A_ = U("A"); idx_ = U("idx"); dang_ = U("dang"); cnt_ = U("cnt");
    safe_ = U("safe"); dist_ = U("dist"); act_ = U("act"); pooled_ = U("pooled"); argmax_ = U("argmax");
    perm_ = U("perm"); host_dist_ = U("host_dist");
    ctrl_w_ = U("ctrl_w"); f_edge_ = (int)I("f_edge"); f_node_ = (int)I("f_node"); ctrl_v_ = U("ctrl_v");
    cbf_w_ = U("cbf_w"); f_fwd_ = (int)I("f_fwd"); cbf_rm_ = U("cbf_rm"); cbf_v_ = U("cbf_v");
    hbuf_ = U("hbuf"); hmask_ = U("hmask"); src_ = U("src"); nev_ = U("nev");
    r2_train_ = F("r2_train"); ttc_train_ = F("ttc_train"); r2_check_ = F("r2_check"); ttc_check_ = F("ttc_check");
    dt_ = F("dt"); obs_r_ = F("obs_r"); sqrt3_ = F("sqrt3"); dist_thr_ = F("dist_thr"); dist_eps_ = F("dist_eps");
    done_thr_ = F("done_thr");
    check_ = (int)I("check_every");
    noise_key_ = U("noise_key"); noise_prob_ = F("noise_prob"); noise_scale_ = F("noise_scale");
    scan_ws_ = U("scan_ws"); scan_ws_env_ = I("scan_ws_env");
    apw_ = (int)I("apw");
    small_ctl_ = U("small_ctl"); small_apw_ = (int)I("small_apw"); knn_tail_ = (int)I("knn_tail");
    small_stamps_ = c.contains("small_stamps") ? U("small_stamps") : 0;
    // the node MLP's activations per step (T, B*N, node_act_bytes), kept for the cooperative node
    // backward (0 = not kept)
    acts_ = c.contains("node_acts") ? U("node_acts") : 0;
    act_bytes_ = c.contains("node_act_bytes") ? I("node_act_bytes") : 0;
    if (small_ctl_) {
      chk(hipHostMalloc((void**)&small_res_, 2 * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
      small_res_[0] = small_res_[1] = 0;
      chk(hipHostGetDevicePointer((void**)&small_res_dev_, small_res_, 0), "hipHostGetDevicePointer");
    }
    // early-stop publication (ctrl.hip publish_step): per-step workgroup counters on the device,
    // the per-env sums and a flag per step in host-coherent memory
    publish_ = c.contains("publish") ? (int)I("publish") : 0;
    poll_query_ms_ = c.contains("poll_query_ms") ? (int)I("poll_query_ms") : 100;
    if (publish_) {
      const size_t nd = (size_t)Tmax_ * B_, bytes = nd * sizeof(unsigned long long) + (size_t)Tmax_ * sizeof(unsigned);
      chk(hipHostMalloc((void**)&pub_host_, bytes, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
      std::memset(pub_host_, 0, bytes);
      chk(hipHostGetDevicePointer((void**)&pub_dev_, pub_host_, 0), "hipHostGetDevicePointer");
      chk(hipMalloc((void**)&pub_ctr_, (size_t)Tmax_ * sizeof(unsigned)), "hipMalloc");
      chk(hipMemset(pub_ctr_, 0, (size_t)Tmax_ * sizeof(unsigned)), "hipMemset");   // once: kernels re-arm them
    }
    if (check_ < 1) check_ = 1;
    if (B_ < 1|| N_ < 1 || Nn_ < N_ || K_ < 1 || K_ > 16 || (D_ != 2 && D_ != 3) || Tmax_ < 1 || resort_ < 1)
      throw std::invalid_argument("RolloutDriver: bad dimensions");
    ev_copy_.resize(Tmax_);
    for (auto& e : ev_copy_) chk(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    // stream -> stream dependencies on one device: a device-scope release is enough (the default
    // system-scope fence writes back / invalidates caches for host visibility and stalls the
    // queue behind it); the copy-completion events the host waits on keep the system fence
    const unsigned fork_flags = hipEventDisableTiming | (c["fork_device_scope"].cast<int>() ? hipEventReleaseToDevice : 0u);
    chk(hipEventCreateWithFlags(&ev_main_, fork_flags), "hipEventCreate");
    chk(hipEventCreateWithFlags(&ev_side_, fork_flags), "hipEventCreate");
  }
  ~RolloutDriver() {
    for (auto e : ev_copy_) (void)hipEventDestroy(e);
    (void)hipEventDestroy(ev_main_);
    (void)hipEventDestroy(ev_side_);
    if (small_res_) (void)hipHostFree(small_res_);
    if (pub_host_) (void)hipHostFree(pub_host_);
    if (pub_ctr_) (void)hipFree(pub_ctr_);
  }
  RolloutDriver(const RolloutDriver&) = delete;
  RolloutDriver& operator=(const RolloutDriver&) = delete;

  // Returns (T, tail_scanned): T valid steps; tail_scanned = the scan of s_T was issued (the
  // early-stopped case, where step T's scan ran before the break).
  std::pair<int, bool> run(u64 stream, u64 hstream, u64 copy_stream, bool early_stop) {
    hipStream_t st = ST(stream), hs = ST(hstream), cs = ST(copy_stream);
    const volatile unsigned long long* hd = P<const volatile unsigned long long>(host_dist_);
    int T = Tmax_;
    bool tail = false;
    // published early stop: the controller kernels hand the per-env sums to the host (no marker)
    const bool pub = publish_ && early_stop;
    if (pub) {
      ++gen_;      // the per-step counters are zero: set at allocation, re-armed by the last workgroup
      hd = pub_host_;
    }
    for (int t = 0; t < Tmax_; ++t) {
      scan_step(t, st);
      ctrl_step(t, st, pub);
      // ONE marker per step on the compute queue (each marker stalls the queue behind it for
      // ~6 us: the next dispatch waits for its completion signal); both side queues wait on it
      if (overlap_ || (early_stop && !pub)) chk(hipEventRecord(ev_main_, st), "hipEventRecord");
      // CBF h of the previous step's main slots on the side stream (one step late: the slice
      // of a step beyond the early stop is never issued)
      if (overlap_ && t >= 1) {
        chk(hipStreamWaitEvent(hs, ev_main_, 0), "hipStreamWaitEvent");
        hfwd_slice(t - 1, hs);
      }
      if (early_stop) {
        if (!pub) {
          chk(hipStreamWaitEvent(cs, ev_main_, 0), "hipStreamWaitEvent");
          chk(hipMemcpyAsync(P<unsigned long long>(host_dist_) + (long)t * B_, P<const unsigned long long>(dist_) + (long)t * B_,
                             sizeof(unsigned long long) * B_, hipMemcpyDeviceToHost, cs), "hipMemcpyAsync");
          chk(hipEventRecord(ev_copy_[t], cs), "hipEventRecord");
        }
        // host check every check_every steps (small scenes: a step's kernels take less than
        // the host round trip, so checking every step would leave the GPU idle)
        if (t >= 1 && (t % check_ == 0)) {
          if (pub) wait_published(t - 1, st);
          else chk(hipEventSynchronize(ev_copy_[t - 1]), "hipEventSynchronize");
          const int Tf = first_done(hd, t - 1);
          if (Tf > 0) {
            // every env was done after step Tf-1: the trajectory is steps 0..Tf-1; step Tf's
            // scan already gave the kNN graph / safety of s_Tf; later steps are unused
            T = Tf;
            tail = true;
            break;
          }
        }
      }
    }
    if (early_stop && !tail && check_ > 1 && Tmax_ >= 2) {
      // steps after the last strided check: same horizon as a check after every step
      if (pub) wait_published(Tmax_ - 2, st);
      else chk(hipEventSynchronize(ev_copy_[Tmax_ - 2]), "hipEventSynchronize");
      const int Tf = first_done(hd, Tmax_ - 2);
      if (Tf > 0) {
        T = Tf;
        tail = true;
      }
    }
    if (overlap_) {
      if (!tail) {
        // the side stream already waits on the marker after ctrl_fwd(T-1) unless T == 1
        if (T == 1) chk(hipStreamWaitEvent(hs, ev_main_, 0), "hipStreamWaitEvent");
        hfwd_slice(T - 1, hs);
      }
      chk(hipEventRecord(ev_side_, hs), "hipEventRecord");     // join the side stream
      chk(hipStreamWaitEvent(st, ev_side_, 0), "hipStreamWaitEvent");
    }
    return {T, tail};     // converted to a tuple after the GIL is re-acquired
  }

  // Executable graphs of the post-rollout work per horizon (index T; 0: none), captured by the
  // engine (hip_engine.py _capture_bwd): run_small(..., launch_graph) launches graph T as soon as
  // the horizon arrives, without a return to Python in between.
  void set_bwd_graphs(std::vector<u64> execs) { bwd_execs_ = std::move(execs); }

  // Persistent small-scene rollout (ctrl.hip rollout_small_kernel): the whole rollout in one
  // launch, early stop decided on the device; returns (T, true, launched) -- the kernel also scanned
  // s_T; launched: the registered graph of horizon T was launched on `stream`.
  // s0 / g0 (optional): the scenario's start states (B, N, 2D) and goals (B, N, D), loaded by the
  // kernel itself.
  std::tuple<int, bool, bool> run_small(u64 stream, bool early_stop, bool launch_graph, u64 s0, u64 g0) {
    if (!small_ctl_) throw std::runtime_error("RolloutDriver: no small-scene control buffer");
    hipStream_t st = ST(stream);
    int* ctl = P<int>(small_ctl_);
    mb::RolloutSmallArgs a{};
    mb::CtrlArgs& c = a.c;
    c.dim = D_;
    c.S = S_at(0); c.s_env = Nn_;
    c.G = P<const float>(G_);
    c.B = B_; c.N = N_; c.K = K_;
    c.wpack = P<const h16>(ctrl_w_); c.f_edge = f_edge_; c.f_node = f_node_; c.wvec = P<const float>(ctrl_v_);
    c.A = P<float>(A_);
    c.dist_sum = P<unsigned long long>(dist_); c.act_sum = P<unsigned long long>(act_);
    c.noise_key = P<const unsigned long long>(noise_key_); c.noise_prob = noise_prob_; c.noise_scale = noise_scale_;
    c.dt = dt_; c.obs_r = obs_r_; c.sqrt3 = sqrt3_;
    c.pooled = P<h16>(pooled_); c.argmax = P<uint8_t>(argmax_);
    c.apw = small_apw_;
    c.stamps = reinterpret_cast<unsigned long long*>(small_stamps_);   // diagnostics builds only (else 0)
    c.acts = P<unsigned char>(acts_); c.na_env = N_;     // per-step views offset in the kernel
    a.idx = P<int>(idx_); a.dang = P<uint8_t>(dang_); a.cnt = P<float>(cnt_);
    a.safe = safety_ ? P<float>(safe_) : nullptr;
    a.Nn = Nn_; a.Tmax = Tmax_; a.knn_tail = knn_tail_;
    a.r2_train = r2_train_; a.ttc_train = ttc_train_; a.r2_check = r2_check_; a.ttc_check = ttc_check_;
    a.done_thr = early_stop ? done_thr_ : -INFINITY;
    a.ctl = ctl;      // zero at allocation; the kernel's last workgroup re-arms it
    a.res = small_res_dev_;
    a.res_gen = (int)++small_gen_;
    a.s0 = P<const float>(s0); a.g0 = P<const float>(g0);
    if ((s0 == 0) != (g0 == 0)) throw std::invalid_argument("run_small: s0 and g0 go together");
    chk((prec_ == 2 ? mb_rollout_small_x3 : prec_ == 1 ? mb_rollout_small_f16 : mb_rollout_small)(&a, st), "rollout_small");
    // the horizon arrives in host-coherent memory when the last workgroup finishes: poll it (a
    // stream synchronisation added a memset, a read-back copy and the blocking wake-up to every
    // iteration of the small configurations)
    const volatile int* res = small_res_;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned long n = 0; __atomic_load_n(&res[1], __ATOMIC_ACQUIRE) != a.res_gen; ++n) {
      if ((n & 4095) == 4095) {
        const auto dt = std::chrono::steady_clock::now() - t0;
        if (dt >= std::chrono::milliseconds(poll_query_ms_)) {
          const hipError_t e = hipStreamQuery(st);
          if (e != hipSuccess && e != hipErrorNotReady) chk(e, "rollout_small stream");
          // the stream drained without the flag: the launch did not run (never spin forever)
          if (e == hipSuccess && __atomic_load_n(&res[1], __ATOMIC_ACQUIRE) != a.res_gen)
            throw std::runtime_error("RolloutDriver: rollout_small finished without publishing its horizon");
        }
        if (dt > std::chrono::seconds(60)) throw std::runtime_error("RolloutDriver: rollout_small horizon not published");
      }
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
    }
    const int T = res[0];
    bool launched = false;
    if (launch_graph && T >= 1 && T < (int)bwd_execs_.size() && bwd_execs_[T]) {
      chk(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(static_cast<uintptr_t>(bwd_execs_[T])), st), "hipGraphLaunch");
      launched = true;
    }
    return {T, true, launched};
  }

 private:
  // Smallest T' (1 <= T' <= t+1) such that every env was done after step T'-1 (env b is done
  // from the first step q_b whose mean goal distance is below the threshold: T' = max_b q_b + 1),
  // or 0 if some env is not done by step t. Checking after every step and breaking at the first
  // hit gives the same T'.
  int first_done(const volatile unsigned long long* hd, int t) const {
    int last = -1;
    for (int b = 0; b < B_; ++b) {
      int q = 0;      // same float arithmetic as rollout_stats_kernel
      while (q <= t && !((float)((double)hd[(long)q * B_ + b] / mb::FX_DIST) / (float)N_ < done_thr_)) ++q;
      if (q > t) return 0;
      if (q > last) last = q;
    }
    return last + 1;
  }

  const float4* S_at(int t) const { return P<const float4>(S_) + (long)t * B_ * Nn_ * (W_ / 4); }

  // Waits until the controller kernel of step t has published its per-env sums (flag == this
  // rollout's generation). Polls host-coherent memory; a stream error or a minute without the
  // flag raises instead of spinning forever.
  void wait_published(int t, hipStream_t st) const {
    const unsigned* flag = reinterpret_cast<const unsigned*>(pub_host_ + (size_t)Tmax_ * B_) + t;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned long n = 0; __atomic_load_n(flag, __ATOMIC_ACQUIRE) != gen_; ++n) {
      if ((n & 4095) == 4095) {
        // the stream-error probe only after poll_query_ms_ of waiting (a step publishes within a
        // millisecond): hipStreamQuery on a busy stream enqueues a marker, and the marker stalled
        // the queue behind it -- the ~6 us gap after every controller step (trace median 5.66 ->
        // 0 us, headline -0.05 ms, profiles/r5_b8/; MACBF_POLL_QUERY_MS=0: probe every 4096 polls)
        const auto dt = std::chrono::steady_clock::now() - t0;
        if (dt >= std::chrono::milliseconds(poll_query_ms_)) {
          const hipError_t e = hipStreamQuery(st);
          if (e != hipSuccess && e != hipErrorNotReady) chk(e, "rollout stream");
        }
        if (dt > std::chrono::seconds(60))
          throw std::runtime_error("RolloutDriver: early-stop flag of step " + std::to_string(t) + " not published");
      }
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
    }
  }

  void scan_step(int t, hipStream_t st) {
    if (t % resort_ == 0) {
      mb::CellSortArgs c{};
      c.S = S_at(t); c.s_env = Nn_; c.B = B_; c.N = Nn_; c.L = L_; c.perm = P<int>(perm_); c.rec = W_ / 4;
      chk(mb_cell_sort(&c, st), "cell_sort");
    }
    mb::ScanArgs a{};
    a.S = S_at(t); a.s_env = Nn_; a.perm = P<const int>(perm_);
    a.B = B_; a.N = N_; a.K = K_; a.Nn = Nn_; a.dim = D_;
    const long nk = (long)N_ * K_;
    a.idx = P<int>(idx_) + (long)t * B_ * nk; a.i_env = nk;
    a.dang = P<uint8_t>(dang_) + (long)t * B_ * nk;
    a.cnt = P<float>(cnt_) + (long)t * B_ * 2; a.c_env = 2;
    a.safe = safety_ ? P<float>(safe_) + (long)t * B_ : nullptr; a.sf_env = 1;
    a.r2_train = r2_train_; a.ttc_train = ttc_train_; a.r2_check = r2_check_; a.ttc_check = ttc_check_;
    a.do_knn = 1; a.do_safety = safety_;
    a.prev_idx = t > 0 ? P<const int>(idx_) + (long)(t - 1) * B_ * nk : nullptr; a.pi_env = nk;
    a.ws = P<float4>(scan_ws_); a.ws_env = scan_ws_env_;
    chk(mb_scan(&a, st), "scan");
  }

  void ctrl_step(int t, hipStream_t st, bool pub = false) {
    mb::CtrlArgs a{};
    if (pub) {
      a.pub_ctr = pub_ctr_ + t;
      a.pub_dist = pub_dev_ + (long)t * B_;
      a.pub_flag = reinterpret_cast<unsigned*>(pub_dev_ + (size_t)Tmax_ * B_) + t;
      a.pub_gen = gen_;
    }
    a.dim = D_;
    a.S = S_at(t); a.s_env = Nn_;
    a.G = P<const float>(G_);
    const long nk = (long)N_ * K_;
    a.idx = P<const int>(idx_) + (long)t * B_ * nk; a.i_env = nk;
    a.acts = acts_ ? P<unsigned char>(acts_) + (long)t * B_ * N_ * act_bytes_ : nullptr; a.na_env = N_;
    a.B = B_; a.N = N_; a.K = K_;
    a.wpack = P<const h16>(ctrl_w_); a.f_edge = f_edge_; a.f_node = f_node_; a.wvec = P<const float>(ctrl_v_);
    a.A = P<float>(A_) + (long)t * B_ * N_ * D_; a.a_env = N_;
    a.Snext = const_cast<float4*>(S_at(t + 1)); a.sn_env = Nn_;
    a.dist_sum = P<unsigned long long>(dist_) + (long)t * B_; a.d_env = 1;
    a.act_sum = P<unsigned long long>(act_) + (long)t * B_; a.ac_env = 1;
    a.noise = nullptr; a.n_env = 0;
    a.noise_key = P<const unsigned long long>(noise_key_); a.noise_prob = noise_prob_; a.noise_scale = noise_scale_;
    a.noise_t = t;
    a.dt = dt_; a.obs_r = obs_r_; a.sqrt3 = sqrt3_;
    a.pooled = P<h16>(pooled_) + (long)t * B_ * N_ * prow_; a.p_env = (long)N_ * prow_;
    a.argmax = P<uint8_t>(argmax_) + (long)t * B_ * N_ * 128; a.am_env = (long)N_ * 128;
    a.apw = apw_;
    chk((prec_ == 2 ? mb_ctrl_fwd_x3 : prec_ == 1 ? mb_ctrl_fwd_f16 : mb_ctrl_fwd)(&a, num_cu_, st), "ctrl_fwd");
  }

  // CBF h of the main slots of step t, evaluations [t*BNK, (t+1)*BNK), on the side stream
  void hfwd_slice(int t, hipStream_t hs) {
    mb::CbfFwdArgs a{};
    a.dim = D_;
    const long bnk = (long)B_ * N_ * K_;
    a.S = P<const float4>(S_); a.s_env = Nn_; a.s_step = (long)B_ * Nn_;
    a.idx = P<const int>(idx_); a.idx1 = a.idx; a.src = P<const int>(src_); a.nev = P<const int>(nev_);
    a.B = B_; a.T = t + 1; a.N = N_; a.K = K_; a.two = 1;
    a.wpack = P<const h16>(cbf_w_); a.f_fwd = f_fwd_; a.wrm = P<const h16>(cbf_rm_);
    a.wvec = P<const float>(cbf_v_);
    a.h_out = P<float>(hbuf_); a.mask_out = P<uint8_t>(hmask_);
    a.obs_r = obs_r_; a.dist_thr = dist_thr_; a.dist_eps = dist_eps_;
    a.u_begin = (unsigned)(t * bnk); a.u_end = (unsigned)((t + 1) * bnk);
    chk((prec_ == 2 ? mb_cbf_hfwd_x3 : prec_ == 1 ? mb_cbf_hfwd_f16 : mb_cbf_hfwd)(&a, hfwd_blocks_, hs), "cbf_hfwd");
  }

  int B_, N_, Nn_, K_, D_, W_, Tmax_, num_cu_, prec_, prow_, resort_, safety_, overlap_, hfwd_blocks_, check_, apw_;
  int publish_ = 0;
  unsigned gen_ = 0;
  int poll_query_ms_ = 0;
  unsigned long long* pub_host_ = nullptr;   // host view: [Tmax][B] sums, then [Tmax] flags
  unsigned long long* pub_dev_ = nullptr;    // the same memory, device view
  unsigned* pub_ctr_ = nullptr;              // [Tmax] per-step workgroup counters (device)
  float L_;
  u64 S_, G_, A_, idx_, dang_, cnt_, safe_, dist_, act_, pooled_, argmax_, perm_, host_dist_;
  u64 ctrl_w_, ctrl_v_, cbf_w_, cbf_rm_, cbf_v_, hbuf_, hmask_, src_, nev_, noise_key_;
  float noise_prob_, noise_scale_;
  u64 scan_ws_;
  long scan_ws_env_;
  u64 small_ctl_ = 0, small_stamps_ = 0, acts_ = 0;
  long act_bytes_ = 0;
  int small_apw_ = 0, knn_tail_ = 0;
  std::vector<u64> bwd_execs_;
  int* small_res_ = nullptr;                 // host-coherent [T, flag] of the persistent rollout
  int* small_res_dev_ = nullptr;             // its device view
  unsigned small_gen_ = 0;
  int f_edge_, f_node_, f_fwd_;
  float r2_train_, ttc_train_, r2_check_, ttc_check_, dt_, obs_r_, sqrt3_, dist_thr_, dist_eps_, done_thr_;
  std::vector<hipEvent_t> ev_copy_;
  hipEvent_t ev_main_ = nullptr, ev_side_ = nullptr;
};

// Native BPTT driver: the reverse-time loop of the controller backward (hand-derived adjoints
// of train.py:58-103's autograd through the rollout). Per step t = T-1..0:
//   ctrl_node_bwd(t)  <- G_{t+1} (dS_T for the last step)
//   ctrl_edge_bwd(t)
//   node_combine(t)   -> G_t
// over the engine's persistent time-major buffers (pointer offsets validated once in Python).
// Three dependent launches per step: the loop is GPU-bound at 1024 x 64 agents but host-bound
// for small scenes (BASELINE config #2: 32 agents), where Python paid ~15 us per launch.
class BpttDriver {
 public:
  explicit BpttDriver(py::dict c) {
    auto I = [&](const char* k) { return c[k].cast<long>(); };
    auto F = [&](const char* k) { return c[k].cast<float>(); };
    auto U = [&](const char* k) { return c[k].cast<u64>(); };
    B_ = (int)I("B"); N_ = (int)I("N"); Nn_ = (int)I("Nn"); K_ = (int)I("K"); D_ = (int)I("D");
    R_ = D_ == 2 ? 1 : 2;
    Tmax_ = (int)I("Tmax"); prec_ = (int)I("prec"); prow_ = prec_ == 2 ? 256 : 128; nb_node_ = (int)I("nb_node"); nb_edge_ = (int)I("nb_edge");
    qsplit_ = (int)I("qsplit");
    pooled_ = U("pooled"); S_ = U("S"); G_ = U("G"); A_ = U("A"); dS_ = U("dS"); Gb_ = U("Gb"); valid_ = U("valid");
    idx_ = U("idx"); argmax_ = U("argmax"); rptr_ = U("rptr"); redges_ = U("redges");
    wrm_ = U("ctrl_rm"); o1_ = (int)I("o_w1"); o2_ = (int)I("o_w2"); o3_ = (int)I("o_w3"); o4_ = (int)I("o_w4");
    wvec_ = U("ctrl_v"); act_scale_ = U("act_scale"); dP_ = U("dP"); ego_ = U("ego"); dEc_ = U("dEc");
    part_node_ = U("part_node"); part_edge_ = U("part_edge");
    wpack_ = U("ctrl_w"); f_ew1f_ = (int)I("f_ew1f"); f_ew2tn_ = (int)I("f_ew2tn");
    dt_ = F("dt"); sqrt3_ = F("sqrt3");
    node_chunk_ = (int)I("node_chunk");
    // per-step slab rows (small grids): step t's node / edge workgroups write rows (T-1-t) x grid
    // of the slabs instead of accumulating into one row per workgroup
    step_rows_ = c.contains("step_rows") ? (int)I("step_rows") : 0;
    acts_ = c.contains("node_acts") ? U("node_acts") : 0;
    act_bytes_ = c.contains("node_act_bytes") ? I("node_act_bytes") : 0;
    node_part_ = c.contains("node_part") ? I("node_part") : 0;
    edge_part_ = c.contains("edge_part") ? I("edge_part") : 0;
    if (step_rows_ && (node_part_ <= 0 || edge_part_ <= 0))
      throw std::invalid_argument("BpttDriver: step_rows needs the slab row sizes");
    fused_ = c.contains("fused_step") ? (int)I("fused_step") : 0;
    if (fused_ && (node_chunk_ != 32 || nb_node_ != nb_edge_))
      throw std::invalid_argument("BpttDriver: the fused step needs 32-agent chunks and one grid");
    gscale_ = c.contains("gscale") ? U("gscale") : 0;   // fp16: device loss scale (or 0)
    ew16_ = c.contains("ctrl_w16") ? U("ctrl_w16") : 0;   // K = 12: 16x16x32 edge backward fragments
    nw16_ = c.contains("node_rm16") ? U("node_rm16") : 0;  // 128-agent chunks: 16x16x32 node backward images
    if (nw16_ && (node_chunk_ != 128 || fused_))
      throw std::invalid_argument("BpttDriver: the 16x16x32 node backward needs 128-agent chunks");
    if (B_ < 1 || N_ < 1 || Nn_ < N_ || K_ < 1 || K_ > 16 || (D_ != 2 && D_ != 3) || Tmax_ < 1 || nb_node_ < 1 ||
        nb_edge_ < 1)
      throw std::invalid_argument("BpttDriver: bad dimensions");
  }

  // use_acts: this iteration's rollout kept the node activations (RolloutDriver with node_acts)
  void run(int T, float act_coef, u64 stream, bool use_acts) {
    if (T < 1 || T > Tmax_) throw std::invalid_argument("BpttDriver: T out of range");
    hipStream_t st = ST(stream);
    const long BN = (long)B_ * N_;
    const long nk = (long)N_ * K_;
    for (int t = T - 1; t >= 0; --t) {
      const float4* Gn = P<const float4>(dS_) + (long)T * BN * R_;       // t = T-1: the direct terms dS_T
      const float4* St = P<const float4>(S_) + (long)t * B_ * Nn_ * R_;
      mb::CtrlNodeBwdArgs na{};
      mb::CtrlEdgeBwdArgs ea{};
      {
        mb::CtrlNodeBwdArgs& a = na;
        a.dim = D_;
        a.pooled = P<const h16>(pooled_) + (long)t * BN * prow_; a.p_env = (long)N_ * prow_;
        a.S = St; a.s_env = Nn_;
        a.G = P<const float>(G_); a.A = P<const float>(A_) + (long)t * BN * D_; a.a_env = N_;
        a.Gn = Gn; a.gn_env = N_;
        a.valid = P<const uint8_t>(valid_) + (long)t * B_; a.v_env = 1;
        a.B = B_; a.N = N_;
        a.wrm = P<const h16>(wrm_); a.o_w1 = o1_; a.o_w2 = o2_; a.o_w3 = o3_; a.o_w4 = o4_;
        a.wvec = P<const float>(wvec_); a.act_coef = act_coef; a.act_scale = P<const float>(act_scale_);
        a.gscale = P<const float>(gscale_);
        a.dt = dt_; a.sqrt3 = sqrt3_;
        a.dP = P<h16>(dP_); a.dp_env = (long)N_ * prow_; a.ego = P<float4>(ego_); a.partial = P<float>(part_node_);
        a.init = t == T - 1;     // the first step of the reverse loop writes the slabs
        if (step_rows_) {
          a.partial += (long)(T - 1 - t) * nb_node_ * node_part_;
          a.init = 1;
        }
        a.chunk = node_chunk_;
        a.acts = (use_acts && acts_) ? P<const unsigned char>(acts_) + (long)t * BN * act_bytes_ : nullptr;
        a.na_env = N_;
        a.wrm16 = P<const h16>(nw16_);
        a.K = K_;
        if (t < T - 1) {
          // fused BPTT combine: G_{t+1} from step t+1's records (dS, ego, dEc, graph t+1, G_{t+2})
          const long t1 = t + 1;
          a.cdS = P<const float4>(dS_) + t1 * BN * R_; a.cds_env = N_;
          // dEc is double-buffered by step parity: step t+1's edge records sit in buffer (t+1)&1
          // while step t's edge phase writes buffer t&1 (the fused launch overlaps the two)
          a.cego = P<const float4>(ego_); a.cdEc = P<const float4>(dEc_) + (t1 & 1) * BN * K_ * R_;
          a.cptr = P<const int>(rptr_) + t1 * B_ * (Nn_ + 1); a.cptr_env = Nn_ + 1;
          a.cedges = P<const int>(redges_) + t1 * B_ * nk; a.cedges_env = nk;
          a.cGn = (t1 == T - 1 ? P<const float4>(dS_) + (long)T * BN * R_ : P<const float4>(Gb_) + (t1 + 1) * BN * R_);
          a.cgn_env = N_;
          a.cGout = P<float4>(Gb_) + t1 * BN * R_; a.cgo_env = N_;
        }
      }
      {
        mb::CtrlEdgeBwdArgs& a = ea;
        a.dim = D_;
        a.S = St; a.s_env = Nn_;
        a.idx = P<const int>(idx_) + (long)t * B_ * nk; a.i_env = nk;
        a.argmax = P<const uint8_t>(argmax_) + (long)t * BN * 128; a.am_env = (long)N_ * 128;
        a.dP = P<const h16>(dP_); a.dp_env = (long)N_ * prow_;
        a.B = B_; a.N = N_; a.K = K_;
        a.wpack = P<const h16>(wpack_); a.f_ew1f = f_ew1f_; a.f_ew2tn = f_ew2tn_;
        a.dEc = P<float4>(dEc_) + (long)(t & 1) * BN * K_ * R_; a.de_env = nk; a.partial = P<float>(part_edge_);
        a.qsplit = qsplit_;
        a.init = t == T - 1;
        if (step_rows_) {
          a.partial += (long)(T - 1 - t) * nb_edge_ * edge_part_;
          a.init = 1;
        }
        a.w16 = fused_ ? nullptr : P<const h16>(ew16_);   // (the fused step keeps its own edge phase)
      }
      if (fused_) {      // node + edge backward of the same 32-agent chunks in one launch
        chk((prec_ == 2 ? mb_ctrl_bwd_step_x3 : prec_ == 1 ? mb_ctrl_bwd_step_f16 : mb_ctrl_bwd_step)(&na, &ea, nb_node_, st),
            "ctrl_bwd_step");
      } else {
        chk((prec_ == 2 ? mb_ctrl_node_bwd_x3 : prec_ == 1 ? mb_ctrl_node_bwd_f16 : mb_ctrl_node_bwd)(&na, nb_node_, st),
            "ctrl_node_bwd");
        chk((prec_ == 2 ? mb_ctrl_edge_bwd_x3 : prec_ == 1 ? mb_ctrl_edge_bwd_f16 : mb_ctrl_edge_bwd)(&ea, nb_edge_, st),
            "ctrl_edge_bwd");
      }
      // (no combine launch: the next step's node backward forms G_t in its prologue; G_0 = dL/ds_0
      // is not needed -- s_0 is sampled, not a function of the weights)
    }
  }

 private:
  int B_, N_, Nn_, K_, D_, R_, Tmax_, prec_, prow_, nb_node_, nb_edge_, qsplit_, node_chunk_ = 0, fused_ = 0;
  int step_rows_ = 0;
  long node_part_ = 0, edge_part_ = 0, act_bytes_ = 0;
  u64 acts_ = 0;
  u64 pooled_, S_, G_, A_, dS_, Gb_, valid_, idx_, argmax_, rptr_, redges_, wrm_, wvec_, act_scale_, dP_, ego_, dEc_;
  u64 part_node_, part_edge_, wpack_, gscale_ = 0, ew16_ = 0, nw16_ = 0;
  int o1_, o2_, o3_, o4_, f_ew1f_, f_ew2tn_;
  float dt_, sqrt3_;
};

}  // namespace

void register_runtime(py::module& m) {
  py::class_<BpttDriver>(m, "BpttDriver")
      .def(py::init<py::dict>())
      .def("run", &BpttDriver::run, py::arg("T"), py::arg("act_coef"), py::arg("stream"), py::arg("use_acts") = false);
  py::class_<RolloutDriver>(m, "RolloutDriver")
      .def(py::init<py::dict>())
      .def("set_bwd_graphs", &RolloutDriver::set_bwd_graphs, py::arg("execs"))
      .def("run_small", &RolloutDriver::run_small, py::arg("stream"), py::arg("early_stop"),
           py::arg("launch_graph") = false, py::arg("s0") = 0, py::arg("g0") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("run", &RolloutDriver::run, py::arg("stream"), py::arg("hstream"), py::arg("copy_stream"),
           py::arg("early_stop"),
           // the loop blocks on hipEventSynchronize: let other Python threads run meanwhile
           py::call_guard<py::gil_scoped_release>());
}
