// Native per-GPU window engine (engine.h) and its small glue kernels.
#include "engine.h"
#include "mislo_packet_kernels.h"

#include <chrono>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>

namespace mislo {

namespace {

#define HIPCHECK(x)                                                                                  \
  do {                                                                                               \
    hipError_t _e = (x);                                                                             \
    if (_e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + \
                                                   " at " #x);                                       \
  } while (0)

#define NCCLCHECK(x)                                                                                        \
  do {                                                                                                      \
    ncclResult_t _r = (x);                                                                                  \
    if (_r != ncclSuccess) throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(_r) + \
                                                    " at " #x);                                             \
  } while (0)

// totals += packet, and the packet stored straight into its pinned host block
__global__ void k_accumulate(const double* __restrict__ packet, double* __restrict__ totals, int n,
                             double* __restrict__ host) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const double v = packet[i];
    totals[i] += v;
    host[i] = v;
  }
}

// The tail of a single-GPU window in one dispatch (it was three: pack, results copy, accumulate):
// the packet from the accumulators -- kept on the device for the prequential refit --, added to
// the run's totals and stored into its pinned host block; the per-incident results block copied
// to its pinned host block.
__global__ __launch_bounds__(256) void k_window_end(const uint32_t* hist, const uint32_t* status,
                                                    const unsigned long long* misc, const unsigned long long* dbg,
                                                    const uint32_t* confusion, const double* stats, const double* count,
                                                    const uint32_t* ring, double* __restrict__ packet,
                                                    double* __restrict__ totals, double* __restrict__ packet_host,
                                                    const uint4* __restrict__ res, uint4* __restrict__ res_host,
                                                    size_t res16) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
  if (t < (size_t)kPacketLen) {
    const double v = packet_value((int)t, hist, status, misc, dbg, confusion, stats, count, ring);
    packet[t] = v;
    totals[t] += v;
    packet_host[t] = v;
  }
  for (size_t i = t; i < res16; i += stride) res_host[i] = res[i];
}

// Small copies between device memory and pinned host memory, by a kernel (loads or stores over
// PCIe). A small hipMemcpyAsync is served by the host through the BAR, which blocks the issuing
// thread until the stream reaches the copy -- for the results D2H the whole window's compute
// (measured: ~480 us per window of host time in submit) -- where a kernel is queued like any
// other launch.
__global__ void k_to_host(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

void to_host(const void* src, void* dst, size_t bytes, hipStream_t st) {
  const size_t n16 = (bytes + 15) / 16;
  const int g = (int)std::min<size_t>(64, (n16 + 255) / 256);
  hipLaunchKernelGGL(k_to_host, dim3(g > 0 ? g : 1), dim3(256), 0, st, static_cast<const uint4*>(src),
                     static_cast<uint4*>(dst), n16);
}

// pinned, device-visible host memory the kernels store into (uncached on the device side)
void* host_block(size_t bytes) {
  void* h = nullptr;
  HIPCHECK(hipHostMalloc(&h, (bytes + 15) & ~size_t(15), hipHostMallocCoherent | hipHostMallocMapped));
  std::memset(h, 0, bytes);
  return h;
}

template <class T>
T* dalloc(size_t n) {
  void* p = nullptr;
  HIPCHECK(hipMalloc(&p, n * sizeof(T) + 64));
  return static_cast<T*>(p);
}

hipEvent_t mk_event(bool timing) {
  hipEvent_t e;
  HIPCHECK(hipEventCreateWithFlags(&e, timing ? hipEventDefault : (hipEventDisableTiming | hipEventBlockingSync)));
  return e;
}

}  // namespace

void engine_set_tables(const Tables& t) { set_tables(&t); }

WindowEngine::WindowEngine(const EngineConfig& cfg) : cfg_(cfg) {
  if (cfg.sig_cap <= 0 || cfg.span_cap <= 0 || cfg.group_cap <= 0 || cfg.group_cap > 4096)
    throw std::invalid_argument("capacities out of range");
  if (cfg.sig_cap >= (1 << 27)) throw std::invalid_argument("sig_cap must be < 2^27 (top-3 key packing)");
  nb_ = std::max(2, cfg.n_buffers);
  max_ahead_ = std::min(nb_, std::max(1, cfg.max_ahead));
  if (cfg.user_cap <= 0 || cfg.user_cap > cfg.sig_cap) throw std::invalid_argument("user_cap must be in [1, sig_cap]");
  if (cfg.import_cap < 0 || cfg.xchg_cap < 0 || cfg.halo_ms < 0) throw std::invalid_argument("negative import sizes");
  if (cfg.halo_windows < 1 || cfg.halo_windows >= kMaxGens)
    throw std::invalid_argument("halo_windows must be in [1, 3] (resident generations)");
  gens_ = cfg.halo_ms > 0 ? 1 + cfg.halo_windows : 1;
  if (2LL * gens_ * ((long long)cfg.sig_cap + cfg.import_cap) >= (1LL << 27))
    throw std::invalid_argument("2 x generations x (sig_cap + import_cap) must be < 2^27 (top-3 key packing)");
  HIPCHECK(hipSetDevice(cfg.device));
  set_join_params(cfg.window_ms, cfg.threshold, cfg.fanout, cfg.group_mode);
  alloc();
}

void WindowEngine::set_join_params(double window_ms, double threshold, int fanout, int group_mode) {
  const int64_t ms = 1000000;
  int64_t outer = (int64_t)llround(window_ms * ms);
  if (outer <= 0) outer = 2000 * ms;
  if (outer >= (1LL << 35)) throw std::invalid_argument("window too large for top-3 key packing (< 34 s)");
  jp_.outer_ns = outer;
  const int64_t tw[4] = {outer, 100 * ms, 250 * ms, 500 * ms};
  for (int k = 0; k < 4; ++k) jp_.win_ns[k] = std::min(outer, tw[k]);
  const float cf[4] = {1.0f, 0.9f, 0.8f, 0.65f};
  for (int k = 0; k < 4; ++k) jp_.conf[k] = cf[k];
  jp_.threshold = threshold > 0 ? (float)threshold : 0.7f;
  if (fanout <= 0) fanout = 3;
  if (fanout > 3) throw std::invalid_argument("GPU join keeps at most 3 candidates per span");
  jp_.fanout = fanout;
  jp_.group_mode = group_mode;
  graphs_.clear();  // captured launches hold the old parameters
}

void WindowEngine::alloc() {
  const int64_t S = cfg_.span_cap, G = cfg_.group_cap;
  n_rows_ = cfg_.sig_cap + cfg_.import_cap;  // the join's rows: the window's records + imported rows
  const int64_t N = n_rows_;
  nblk_sig_ = decode_grid((int)N);
  nblk_span_ = decode_grid((int)S);
  // MISLO_ONE_STREAM=1: the window's copies on the compute stream (one HIP stream). With one
  // hardware queue (the agent's GPU_MAX_HW_QUEUES=1) the two streams' commands run in order on
  // that queue anyway, and the copy stream's first use maps another ~173 MB queue save area
  // (tools/rss_probe.py); the bench keeps the two streams (copy / compute overlap on 4 queues).
  const bool one_stream = [] {
    const char* v = getenv("MISLO_ONE_STREAM");
    return v && atoi(v) == 1;
  }();
  HIPCHECK(hipStreamCreateWithFlags(&compute_, hipStreamNonBlocking));
  if (one_stream) copy_ = compute_;
  else HIPCHECK(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking));
  {  // MISLO_SPIN_WAIT=1: wait() polls its event instead of sleeping on it
    const char* v = getenv("MISLO_SPIN_WAIT");
    spin_ = v && atoi(v) == 1;
  }
  {  // MISLO_COPY_STREAMS=2 splits a window's DMA over two streams (measured slower: the
     // second stream's large copy blocks the issuing thread ~0.2 ms per window)
    const char* v = getenv("MISLO_COPY_STREAMS");
    if (v && atoi(v) == 2 && !one_stream) HIPCHECK(hipStreamCreateWithFlags(&copy2_, hipStreamNonBlocking));
    else copy2_ = copy_;
  }
  {
    // The span side of the chain (decode, partition, sort, the probe's work list) on a second
    // stream, overlapping the signal side's decode: on by default where the streams have
    // hardware queues to overlap on (not with MISLO_ONE_STREAM, the one-queue agent);
    // MISLO_SPAN_STREAM=0/1 overrides. At the default priority it measured 0.521-0.526 against
    // 0.539-0.546 ms per window (K = 100, profiles/r5_probe/README.md); a high-priority side
    // stream (MISLO_SPAN_STREAM_PRIO=1, its own hardware-queue pool) measured 0.65.
    const char* v = getenv("MISLO_SPAN_STREAM");
    branch_ = v ? atoi(v) == 1 : !one_stream;
    if (branch_) {
      int lo = 0, hi = 0;
      HIPCHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
      const char* pv = getenv("MISLO_SPAN_STREAM_PRIO");  // 1 = the highest priority
      if (pv && atoi(pv) == 1)
        HIPCHECK(hipStreamCreateWithPriority(&side_, hipStreamNonBlocking, hi));
      else
        HIPCHECK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
      for (hipEvent_t* e : {&ev_fork_, &ev_sigbase_, &ev_spans_})
        HIPCHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
      const char* xv = getenv("MISLO_XCHG_SPAN_SIDE");  // 0: the exchange path's span side in part 2
      xspan_ = !(xv && atoi(xv) == 0);
    }
  }
  // one GPU: the window's tail (packet accumulate, timing) runs on the compute stream; a comm
  // stream of its own exists only with a communicator (init_comm). Every stream backs a
  // hardware queue, and each MI355X queue pins ~173 MB of host memory (its context save area,
  // measured: tools/rss_probe.py), so a single-GPU agent does without it.
  comm_stream_ = compute_;
  // device input block per buffer: [head (counts + labels) | framed ring records | user records | spans]
  const size_t head = (kHeadBytes + 4 * (size_t)G + 63) & ~size_t(63);
  off_kern_ = head;
  off_user_ = (off_kern_ + kern_bytes() + 63) & ~size_t(63);
  off_span_ = off_user_ + 64 * (size_t)cfg_.user_cap;
  in_bytes_ = off_span_ + 64 * (size_t)S;
  for (int b = 0; b < nb_; ++b) {
    in_dev_.push_back(dalloc<uint8_t>(in_bytes_));
    HIPCHECK(hipMemset(in_dev_.back(), 0, in_bytes_));
    void* h = nullptr;
    head_host_.push_back(static_cast<uint8_t*>(host_block(head)));
    staging_.push_back(nullptr);  // pinned staging is allocated on first use (unregistered rings only)
    packet_dev_.push_back(dalloc<double>(kPacketLen));
    HIPCHECK(hipMemset(packet_dev_.back(), 0, kPacketLen * sizeof(double)));
    packet_host_.push_back(static_cast<double*>(host_block(kPacketLen * sizeof(double))));
    h2d_done_.push_back(mk_event(false));
    h2d_part_.push_back(mk_event(false));
    head_done_.push_back(mk_event(false));
    compute_done_.push_back(mk_event(false));
    comm_done_.push_back(mk_event(false));
    t_start_.push_back(mk_event(true));
    t_copy_end_.push_back(mk_event(true));
    t_comp0_.push_back(mk_event(true));
    t_comp1_.push_back(mk_event(true));
    t_end_.push_back(mk_event(true));
  }
  warm_.assign(8 * nb_, false);
  // per-incident results block: [post G*16 f64][gconf G f64][feat G*16 f32][pred G i32][evbits G*16 u32]
  // [sli G*2 u32][app G*2 u32][late G*2 u32]
  const size_t o_gconf = 16 * G * 8, o_feat = o_gconf + G * 8, o_pred = o_feat + 16 * G * 4, o_ev = o_pred + G * 4;
  const size_t o_sli = o_ev + 16 * G * 4;
  res_bytes_ = o_sli + 6 * G * 4;
  for (int b = 0; b < nb_; ++b) {
    res_host_.push_back(static_cast<uint8_t*>(host_block(res_bytes_)));
  }
  for (int b = 0; b < nb_; ++b) {  // per buffer: the comm stream gathers window k's while k+1 computes
    res_dev_.push_back(dalloc<uint8_t>(res_bytes_));
    HIPCHECK(hipMemset(res_dev_.back(), 0, res_bytes_));
  }
  // pod metadata, ring accounting, the trace id -> hash table
  pod_sn_ = dalloc<uint32_t>(kPodRows);
  HIPCHECK(hipMemset(pod_sn_, 0, kPodRows * 4));
  {
    void* h = nullptr;
    HIPCHECK(hipHostMalloc(&h, kPodRows * 4, hipHostMallocDefault));
    std::memset(h, 0, kPodRows * 4);
    pod_host_ = static_cast<uint32_t*>(h);
  }
  ring_state_ = dalloc<uint32_t>(kRsLen);
  trace_hash_ = dalloc<unsigned long long>(kTraceIdRows);
  HIPCHECK(hipMemset(trace_hash_, 0, (size_t)kTraceIdRows * 8));
  // other GPUs' trace rows and the selection of this GPU's; the generations' state
  rows_ = dalloc<int>(16);
  tmax_ = dalloc<unsigned long long>(1);
  HIPCHECK(hipMemset(tmax_, 0, 8));
  remote_n_ = dalloc<uint32_t>(nb_);
  HIPCHECK(hipMemset(remote_n_, 0, nb_ * 4));
  gen_ = dalloc<GenMeta>(1);
  {
    GenMeta g{};
    g.cur = (uint32_t)gens_ - 1;  // the first window's k_gen_begin moves to slot 0
    for (int a = 0; a < kMaxGens; ++a) g.cut[a] = INT64_MAX;
    HIPCHECK(hipMemcpy(gen_, &g, sizeof(g), hipMemcpyHostToDevice));
  }
  sel_cnt_ = dalloc<uint32_t>(1024);
  sel_off_ = dalloc<uint32_t>(1024);
  for (int b = 0; b < nb_; ++b) imp_.push_back(cfg_.import_cap ? dalloc<SigRec>(cfg_.import_cap) : nullptr);
  xstride_ = sizeof(XRec) * (1 + (size_t)cfg_.xchg_cap);  // [24-byte header: row count | XRec rows]
  if (cfg_.xchg_cap) {
    xsend_ = dalloc<uint8_t>(xstride_);
    HIPCHECK(hipMemset(xsend_, 0, xstride_));
    const char* tp = getenv("MISLO_SEL_TWO_PASS");
    if (!(tp && atoi(tp) == 1)) {  // the fused selection's ballot masks (segment 0's decode geometry)
      sel_stride_ = decode_sel_stride(n_rows_);
      sel_mask_ = dalloc<unsigned long long>((size_t)decode_grid(n_rows_) * (size_t)sel_stride_);
    }
  }
  // context table: every id the kernel or the host encoder can assign, HBM-resident
  ctx_tab_ = dalloc<uint32_t>((size_t)kCtxRows * 4);
  HIPCHECK(hipMemset(ctx_tab_, 0, (size_t)kCtxRows * 16));
  totals_ = dalloc<double>(kPacketLen);
  HIPCHECK(hipMemset(totals_, 0, kPacketLen * sizeof(double)));
  stats_acc_ = dalloc<double>(kStatsLen);
  HIPCHECK(hipMemset(stats_acc_, 0, kStatsLen * sizeof(double)));
  p0_ = dalloc<double>(2 * kSlots * 16);  // the Beta prior's table, then the likelihood floor
  HIPCHECK(hipMemset(p0_, 0, 2 * kSlots * 16 * sizeof(double)));
  model_dev_ = dalloc<uint8_t>(sizeof(PosteriorModel));
  HIPCHECK(hipMemset(model_dev_, 0, sizeof(PosteriorModel)));
  app_dev_ = dalloc<AppModel>(1);
  HIPCHECK(hipMemset(app_dev_, 0, sizeof(AppModel)));  // on = 0: no application evidence until set
  for (int i = 0; i < max_ahead_ + 2; ++i) {
    void* h = nullptr;
    HIPCHECK(hipHostMalloc(&h, sizeof(PosteriorModel), hipHostMallocDefault));
    model_host_.push_back(static_cast<uint8_t*>(h));
  }
  g_status_ = dalloc<uint8_t>(N);
  g_part_ = dalloc<PartCodes>(N);
  // other GPUs' rows decode in blocks of their own (<= 7 peers' exchange blocks)
  nblk_imp_ = cfg_.xchg_cap ? decode_grid(7 * cfg_.xchg_cap) : 0;
  g_part_blk_ = dalloc<uint32_t>((size_t)(nblk_sig_ + nblk_imp_) * kKeyTypes * kParts);
  g_part_off_ = dalloc<uint32_t>((size_t)(nblk_sig_ + nblk_imp_) * kKeyTypes * kParts);
  for (int b = 0; b < nb_; ++b) xchg_done_.push_back(mk_event(false));
  g_part_tot_ = dalloc<uint32_t>(kKeyTypes * kParts);
  g_part_base_ = dalloc<uint32_t>((size_t)gens_ * kBaseLen);
  // resident generations: rows, partition lists, list keys and offsets of the last gens_ windows
  g_items_ = dalloc<uint32_t>((size_t)gens_ * kKeyTypes * N);
  g_keys_ = dalloc<KeyTs>((size_t)gens_ * kKeyTypes * N);
  g_rec_ = dalloc<SigRec>((size_t)gens_ * N);
  s_part_ = dalloc<PartCodes>(S);
  s_part_blk_ = dalloc<uint32_t>((size_t)nblk_span_ * kKeyTypes * kParts);
  s_part_off_ = dalloc<uint32_t>((size_t)nblk_span_ * kKeyTypes * kParts);
  s_part_tot_ = dalloc<uint32_t>(kKeyTypes * kParts);
  s_part_base_ = dalloc<uint32_t>(kKeyTypes * kParts + 1);
  s_items_ = dalloc<uint32_t>(kKeyTypes * S);
  s_pre_ = dalloc<PreSpan>((size_t)kKeyTypes * S);
  s_rec_ = dalloc<SpanRec>(S);
  probe_work_ = dalloc<uint32_t>(kProbeWorkLen);
  HIPCHECK(hipMemset(probe_work_, 0, kProbeWorkLen * 4));
  top3_ = dalloc<unsigned long long>(3 * S);
  cnt_ = dalloc<uint32_t>(S);
  attrs_ = dalloc<float>(S * kSlots);
  conf_ = dalloc<float>(S);
  kernel_ms_ = dalloc<float>(S);
  gsum_ = dalloc<unsigned long long>((size_t)kGroupStripes * G * kSlots);
  gcnt_ = dalloc<uint32_t>((size_t)kGroupStripes * G * kSlots);
  hist_ = dalloc<uint32_t>(kSlots * kBuckets);
  status_ = dalloc<uint32_t>(kSlots * 3);
  misc_ = dalloc<unsigned long long>(kPacketMisc);
  dbg_ = dalloc<unsigned long long>(kPacketDbg);
  confusion_ = dalloc<uint32_t>(kMaxDomains * kMaxDomains);
  stats_ = dalloc<double>(32 * 32);
  stats_count_ = dalloc<double>(kMaxDomains);
  HIPCHECK(hipDeviceSynchronize());
}

WindowEngine::~WindowEngine() {
  hipDeviceSynchronize();
  for (auto& kv : graphs_) hipGraphExecDestroy(kv.second);
  for (auto g : graph_defs_) hipGraphDestroy(g);
  if (xcomm_) ncclCommDestroy(xcomm_);
  if (comm_) ncclCommDestroy(comm_);
  auto evs = {&t_copy_end_, &h2d_done_, &h2d_part_, &head_done_, &compute_done_, &comm_done_, &t_start_, &t_comp0_, &t_comp1_, &t_end_};
  for (auto* v : evs)
    for (auto e : *v) hipEventDestroy(e);
  for (auto& r : registered_) hipHostUnregister(const_cast<uint8_t*>(r.first));
  for (auto p : head_host_) hipHostFree(p);
  for (auto p : staging_)
    if (p) hipHostFree(p);
  if (pod_host_) hipHostFree(pod_host_);
  for (auto p : res_all_host_) hipHostFree(p);
  for (auto p : res_all_dev_) hipFree(p);
  for (auto p : imp_)
    if (p) hipFree(p);
  for (auto e : xchg_done_) hipEventDestroy(e);
  for (auto p : packet_host_) hipHostFree(p);
  for (auto p : res_host_) hipHostFree(p);
  for (auto p : model_host_) hipHostFree(p);
  for (auto p : in_dev_) hipFree(p);
  for (auto p : packet_dev_) hipFree(p);
  for (auto p : res_dev_) hipFree(p);
  void* bufs[] = {ctx_tab_, totals_, stats_acc_, p0_, model_dev_, g_status_, g_part_, g_part_blk_, g_part_off_,
                  g_part_tot_, g_part_base_, g_items_, g_rec_, s_part_, s_part_blk_, s_part_off_, s_part_tot_,
                  s_part_base_, s_items_, s_rec_, probe_work_, top3_, cnt_, attrs_, conf_, kernel_ms_, gsum_, gcnt_,
                  hist_, status_, misc_, dbg_, confusion_, stats_, stats_count_, pod_sn_, ring_state_, trace_hash_,
                  rows_, tmax_, remote_n_, sel_cnt_, sel_off_, sel_mask_, xsend_, xrecv_, g_keys_, gen_, s_pre_, app_dev_};
  for (void* p : bufs)
    if (p) hipFree(p);
  if (copy_ && copy_ != compute_) hipStreamDestroy(copy_);
  if (copy2_ && copy2_ != copy_) hipStreamDestroy(copy2_);
  if (compute_) hipStreamDestroy(compute_);
  if (side_) hipStreamDestroy(side_);
  for (hipEvent_t e : {ev_fork_, ev_sigbase_, ev_spans_})
    if (e) hipEventDestroy(e);
  if (comm_stream_ && comm_stream_ != compute_) hipStreamDestroy(comm_stream_);
}

SignalCols WindowEngine::sig_cols() const {
  return SignalCols{g_rec_, g_status_, g_part_, g_items_, g_keys_, g_part_base_, gen_, (int64_t)n_rows_, gens_};
}
SpanCols WindowEngine::span_cols() const { return SpanCols{s_rec_, s_part_}; }

bool WindowEngine::register_host(const void* ptr, size_t bytes) {
  if (!ptr || !bytes) return false;
  if (registered(ptr, bytes)) return true;
  if (hipHostRegister(const_cast<void*>(ptr), bytes, hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  registered_.emplace_back(static_cast<const uint8_t*>(ptr), bytes);
  return true;
}

bool WindowEngine::registered(const void* p, size_t n) const {
  const uint8_t* q = static_cast<const uint8_t*>(p);
  for (const auto& r : registered_)
    if (q >= r.first && q + n <= r.first + r.second) return true;
  return false;
}

// DMA a window's segments of one kind back to back into dst (device); unregistered segments go
// through pinned staging (one host memcpy, then the DMA). Returns the bytes placed.
size_t WindowEngine::dma(const std::vector<Seg>& segs, uint8_t* dst, size_t cap, uint8_t*& staging, size_t& st_off,
                         hipStream_t st) {
  size_t off = 0;
  for (const Seg& s : segs) {
    if (!s.bytes) continue;
    if (off + s.bytes > cap) throw std::invalid_argument("window input exceeds the engine's capacity");
    const void* src = s.ptr;
    if (!registered(s.ptr, s.bytes)) {
      if (!staging) {
        void* h = nullptr;
        HIPCHECK(hipHostMalloc(&h, in_bytes_ - off_kern_, hipHostMallocDefault));
        staging = static_cast<uint8_t*>(h);
      }
      std::memcpy(staging + st_off, s.ptr, s.bytes);
      src = staging + st_off;
      st_off += s.bytes;
      staged_bytes_ += s.bytes;
    } else {
      direct_bytes_ += s.bytes;
    }
    HIPCHECK(hipMemcpyAsync(dst + off, src, s.bytes, hipMemcpyHostToDevice, st));
    off += s.bytes;
  }
  return off;
}

bool WindowEngine::h2d_done(int64_t k) {
  for (hipEvent_t ev : {h2d_done_[k % nb_], h2d_part_[k % nb_]}) {  // both copy streams
    const hipError_t e = hipEventQuery(ev);
    if (e == hipErrorNotReady) return false;
    HIPCHECK(e);
  }
  return true;
}

void WindowEngine::wait_h2d(int64_t k) {
  HIPCHECK(hipEventSynchronize(h2d_done_[k % nb_]));
  HIPCHECK(hipEventSynchronize(h2d_part_[k % nb_]));
}

// This buffer's per-incident result pointers (read by the kernels the parts launch).
void WindowEngine::set_buffer(int b) {
  const int G = cfg_.group_cap;
  uint8_t* r = res_dev_[b];  // this buffer's per-incident results block
  const size_t o_gconf = 16 * (size_t)G * 8, o_feat = o_gconf + (size_t)G * 8, o_pred = o_feat + 16 * (size_t)G * 4;
  const size_t o_ev = o_pred + (size_t)G * 4, o_sli = o_ev + 16 * (size_t)G * 4;
  post_ = reinterpret_cast<double*>(r);
  gconf_ = reinterpret_cast<double*>(r + o_gconf);
  feat_ = reinterpret_cast<float*>(r + o_feat);
  pred_ = reinterpret_cast<int32_t*>(r + o_pred);
  evbits_ = reinterpret_cast<uint32_t*>(r + o_ev);
  sli_ = reinterpret_cast<uint32_t*>(r + o_sli);
  app_ = sli_ + 2 * (size_t)G;
  late_ = sli_ + 4 * (size_t)G;
}

// The head of a window: the accumulators reset, the next generation slot, the window's rows.
void WindowEngine::run_begin(int b, hipStream_t st) {
  set_buffer(b);
  const int* counts = reinterpret_cast<const int*>(in_dev_[b]);
  const int S = cfg_.span_cap, G = cfg_.group_cap;
  FillList fl{};
  auto add = [&](void* p, size_t bytes, uint32_t v) { fl.seg[fl.count++] = FillSeg{(uint32_t*)p, (uint32_t)(bytes / 4), v}; };
  add(hist_, kSlots * kBuckets * 4, 0);
  add(status_, kSlots * 3 * 4, 0);
  add(misc_, kPacketMisc * 8, 0);
  add(dbg_, kPacketDbg * 8, 0);
  add(confusion_, kMaxDomains * kMaxDomains * 4, 0);
  add(stats_, 32 * 32 * 8, 0);
  add(stats_count_, kMaxDomains * 8, 0);
  add(top3_, 3 * (size_t)S * 8, 0xFFFFFFFFu);
  add(cnt_, (size_t)S * 4, 0);
  add(gsum_, (size_t)kGroupStripes * G * kSlots * 8, 0);
  add(gcnt_, (size_t)kGroupStripes * G * kSlots * 4, 0);
  add(sli_, (size_t)G * 6 * 4, 0);  // + the application retrieval counts (app_) and late breaches (late_)
  // + the next generation slot and the halo cut-offs (the finished window's tmax is read before
  // its reset), the ring state, no other GPUs' rows until merged, the window's rows
  launch_window_begin(fl, gen_, tmax_, gens_, (long long)llround(cfg_.halo_ms * 1e6), ring_state_, remote_n_ + b,
                      counts, n_rows_, rows_, st);
}

// The captured part of a window: everything between the DMA and the packet.
// Part 1 of a window: accumulators, definitions, the decode of the window's records and the
// halo it imported; with the GPU exchange, this window's trace-tagged rows for the others.
void WindowEngine::run_part1(int b, hipStream_t st, bool xchg) {
  uint8_t* in = in_dev_[b];
  const int* counts = reinterpret_cast<const int*>(in);
  const int N = n_rows_;
  if (!(xchg && xspan_)) run_begin(b, st);  // else its own launch (submit: part 4)
  else set_buffer(b);
  // the span branch in the one-GPU chain: forked inside the window's graph and joined before the
  // probe. With the exchange, forked inside part 1's graph and joined before the exchange it
  // measured 0.76 against 0.62 ms per window (bench.py --rccl-self); there the span side is a
  // graph of its own on side_ instead (xspan_, submit: parts 4 and 3)
  if (branch_ && !xchg) run_span_branch(b, st);
  const TraceIds tt{trace_hash_, kTraceIdRows};
  launch_ring_defs(in + off_kern_, counts, cfg_.sig_cap, ctx_tab_, kCtxRows, pod_sn_, kPodRows, tt, ring_state_, st);
  const bool fused_sel = xchg && sel_mask_;  // the selection's count and masks left by the decode
  launch_decode_window(in + off_kern_, in + off_user_, counts, rows_, N, imp_[b], ctx_tab_, (int)kCtxRows, tt,
                       ring_state_, tmax_, pod_sn_, kPodRows, sig_cols(), hist_, status_, g_part_blk_, misc_, st, 0, 0, 0,
                       rec_shard_rank(), rec_shard_world(), fused_sel ? sel_cnt_ : nullptr,
                       fused_sel ? sel_mask_ : nullptr, sel_stride_);
  // this window's warn-level trace-tagged rows, as the other GPUs will import them
  if (fused_sel)
    launch_select_masked(sig_cols(), rows_, N, sel_cnt_, sel_off_, sel_mask_, sel_stride_,
                         reinterpret_cast<XRec*>(xsend_ + sizeof(XRec)), reinterpret_cast<uint32_t*>(xsend_),
                         (uint32_t)cfg_.xchg_cap, st, dbg_ + kDbgXchgDropped);
  else if (xchg)
    launch_select(sig_cols(), rows_, counts, N, sel_cnt_, sel_off_, reinterpret_cast<XRec*>(xsend_ + sizeof(XRec)),
                  reinterpret_cast<uint32_t*>(xsend_), (uint32_t)cfg_.xchg_cap, st, dbg_ + kDbgXchgDropped);
}

// Part 2: [the other GPUs' rows] -> partition -> spans -> join (this window's spans x every
// generation's visible rows) -> posterior -> packet.
void WindowEngine::run_part2(int b, int n_groups, bool with_labels, bool learn, hipStream_t st, bool xchg) {
  uint8_t* in = in_dev_[b];
  const int* counts = reinterpret_cast<const int*>(in);
  const int32_t* labels = reinterpret_cast<const int32_t*>(in + kHeadBytes);
  const int N = n_rows_, S = cfg_.span_cap, G = cfg_.group_cap;
  if (xchg) {
    const TraceIds tt{trace_hash_, kTraceIdRows};
    launch_decode_window(in + off_kern_, in + off_user_, counts, rows_, N, imp_[b], ctx_tab_, (int)kCtxRows, tt,
                         ring_state_, tmax_, pod_sn_, kPodRows, sig_cols(), hist_, status_, g_part_blk_, misc_, st,
                         1, nblk_imp_, nblk_sig_, rec_shard_rank(), rec_shard_world());
  }
  const bool branched = branch_ && !xchg;
  // with the span branch: the signal bases are what the branch's probe work list waits for
  hipEvent_t sig_base = branched ? ev_sigbase_ : nullptr;
  // without the span branch: the span side first, so the signal scatter's launch can build the
  // probe's work list next to it (it needs both sides' list offsets); with the exchange and
  // xspan_ the span side ran on side_ next to part 1 (submit: part 3)
  if (!branched && !(xchg && xspan_)) run_spans(b, st);
  const uint32_t* wspan = branched ? nullptr : s_part_base_;
  const JoinParams* wjp = branched ? nullptr : &jp_;
  uint32_t* wlist = branched ? nullptr : probe_work_;
  if (xchg)
    launch_partition_sig(sig_cols(), rows_, N, nblk_sig_ + nblk_imp_, g_part_blk_, g_part_off_, g_part_tot_, st,
                         nblk_sig_, sig_base, wspan, wjp, wlist);
  else
    launch_partition_sig(sig_cols(), rows_, N, nblk_sig_, g_part_blk_, g_part_off_, g_part_tot_, st, 0, sig_base,
                         wspan, wjp, wlist);
  if (branched) {  // the work list needs the signal bases just recorded; then join
    HIPCHECK(hipStreamWaitEvent(side_, ev_sigbase_, 0));
    launch_probe_work(s_part_base_, sig_cols(), jp_, probe_work_, side_);
    HIPCHECK(hipEventRecord(ev_spans_, side_));
    HIPCHECK(hipStreamWaitEvent(st, ev_spans_, 0));  // spans sorted, work list built
  }
  launch_probe(span_cols(), s_items_, s_part_base_, sig_cols(), S, jp_, top3_, cnt_, n_groups, gsum_, gcnt_, dbg_,
               probe_work_, s_pre_, st);
  launch_finalize(counts + 1, S, top3_, cnt_, sig_cols(), span_cols(), jp_, nullptr, attrs_, conf_, kernel_ms_,
                  n_groups, gsum_, gcnt_, feat_, dbg_, st);
  const PosteriorModel* pm = reinterpret_cast<const PosteriorModel*>(model_dev_);
  if (learn)
    launch_posterior_stats(feat_, counts + 2, G, pm, with_labels ? labels : nullptr, post_, pred_, gconf_, evbits_,
                           confusion_, labels, nullptr, stats_, stats_count_, st, app_dev_, app_);
  else
    launch_posterior(feat_, counts + 2, G, pm, with_labels ? labels : nullptr, post_, pred_, gconf_, evbits_,
                     confusion_, st, app_dev_, app_);
  if (!comm_) {  // one GPU: the whole tail here (see k_window_end)
    const size_t res16 = (res_bytes_ + 15) / 16;
    const int g = (int)std::max<size_t>((kPacketLen + 255) / 256, std::min<size_t>(64, (res16 + 255) / 256));
    hipLaunchKernelGGL(k_window_end, dim3(g), dim3(256), 0, st, hist_, status_, misc_, dbg_, confusion_, stats_,
                       stats_count_, ring_state_, packet_dev_[b], totals_, packet_host_[b],
                       reinterpret_cast<const uint4*>(res_dev_[b]), reinterpret_cast<uint4*>(res_host_[b]), res16);
    return;
  }
  hipLaunchKernelGGL(k_pack, dim3((kPacketLen + 255) / 256), dim3(256), 0, st, hist_, status_, misc_, dbg_, confusion_,
                     stats_, stats_count_, ring_state_, packet_dev_[b]);
}

// The span side of the chain: decode, partition, span sort (inputs: the span DMA and the reset
// accumulators only).
void WindowEngine::run_spans(int b, hipStream_t st) {
  uint8_t* in = in_dev_[b];
  const int* counts = reinterpret_cast<const int*>(in);
  const int S = cfg_.span_cap, G = cfg_.group_cap;
  const SpanMap sm{1, sli_, G, cfg_.ttft_slo_ms, cfg_.shard_rank, cfg_.shard_world, gen_, app_, late_};
  launch_decode_spans(in + off_span_, counts + 1, S, span_cols(), s_part_blk_, ctx_tab_, (int)kCtxRows, st, &sm);
  launch_partition(s_part_, counts + 1, S, nblk_span_, s_part_blk_, s_part_off_, s_part_tot_, s_part_base_, s_items_,
                   st);
  launch_span_sort(span_cols(), s_items_, s_part_base_, s_pre_, st);
}

// Fork from `st` (after k_window_begin): the span side on side_. run_part2 continues the branch
// once the signal side's partition bases exist -- the probe work list reads both sides' bases
// and time ranges -- and joins it before the probe (ev_spans_). Native 64-byte spans never read
// the context table, so the branch does not wait for k_ring_defs.
void WindowEngine::run_span_branch(int b, hipStream_t st) {
  HIPCHECK(hipEventRecord(ev_fork_, st));
  HIPCHECK(hipStreamWaitEvent(side_, ev_fork_, 0));
  run_spans(b, side_);
}

// Launch a chain part eagerly, or through its captured graph (captured on the buffer's second
// use; the first use runs eagerly so lazily initialised state is out of the capture).
void WindowEngine::launch_part(int part, int b, int n_groups, bool with_labels, bool learn, bool xchg) {
  auto run = [&] {
    if (part == 0) {  // the whole window in one graph (no exchange)
      run_part1(b, compute_, false);
      run_part2(b, n_groups, with_labels, learn, compute_, false);
    } else if (part == 1) {
      run_part1(b, compute_, xchg);
    } else if (part == 2) {
      run_part2(b, n_groups, with_labels, learn, compute_, xchg);
    } else if (part == 3) {  // the exchange path's span side (xspan_)
      run_spans(b, side_);
    } else {  // part 4: the exchange path's window head (xspan_)
      run_begin(b, compute_);
    }
  };
  hipStream_t cs = part == 3 ? side_ : compute_;  // the stream the part is captured on
  if (!cfg_.use_graphs) return run();
  auto key = std::make_tuple(b * 8 + part, n_groups, with_labels, learn);
  auto it = graphs_.find(key);
  if (it == graphs_.end() && !warm_[b * 8 + part]) {
    run();
    warm_[b * 8 + part] = true;
    return;
  }
  if (it == graphs_.end()) {
    hipGraph_t g;
    HIPCHECK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
    run();
    HIPCHECK(hipStreamEndCapture(cs, &g));
    hipGraphExec_t ex;
    HIPCHECK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    graph_defs_.push_back(g);
    it = graphs_.emplace(key, ex).first;
  }
  HIPCHECK(hipGraphLaunch(it->second, cs));
}

void WindowEngine::submit(int64_t k, const WindowInput& in, bool with_labels, bool learn) {
  const auto t0 = std::chrono::steady_clock::now();
  if (k != submitted_) throw std::invalid_argument("windows must be submitted in order");
  const int n_groups = in.n_groups;
  if (n_groups < 0 || n_groups > cfg_.group_cap) throw std::invalid_argument("n_groups exceeds group capacity");
  size_t kb = 0, ub = 0, sb = 0;
  for (const Seg& s : in.kernel) kb += s.bytes;
  for (const Seg& s : in.user) ub += s.bytes;
  for (const Seg& s : in.spans) sb += s.bytes;
  // what the kernels will assume, checked on the host before anything is queued
  if (in.user_rec != 64 && in.user_rec != 32 && in.user_rec != 24 && in.user_rec != 16)
    throw std::invalid_argument("user records are 64, 32, 24 or 16 bytes");
  if (kb % kRecStride || ub % in.user_rec || sb % 64) throw std::invalid_argument("segments must hold whole records");
  // kernel rows: every slot of every batch record (definitions and pads become holes)
  const size_t n_k = kb / kRecStride * kBatchSlots, n_u = ub / in.user_rec, n_s = sb / 64;
  if (n_k + n_u > (size_t)cfg_.sig_cap || n_u > (size_t)cfg_.user_cap || n_s > (size_t)cfg_.span_cap)
    throw std::invalid_argument("window exceeds the engine's capacity (events / user records / spans)");
  const int b = (int)(k % nb_);
  // host back-pressure: at most max_ahead windows queued beyond the one computing
  const auto tw = std::chrono::steady_clock::now();
  if (k >= max_ahead_) HIPCHECK(hipEventSynchronize(compute_done_[(k - max_ahead_) % nb_]));
  // the pinned head / staging of buffer b were last read by the DMAs of window k - nb
  if (k >= nb_) {
    HIPCHECK(hipEventSynchronize(h2d_done_[b]));
    HIPCHECK(hipEventSynchronize(h2d_part_[b]));
    HIPCHECK(hipEventSynchronize(head_done_[b]));
  }
  wait_us_ += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tw).count();
  const auto td = std::chrono::steady_clock::now();
  int32_t* c = reinterpret_cast<int32_t*>(head_host_[b]);
  std::memset(c, 0, kHeadBytes);
  c[0] = (int32_t)(n_k + n_u);
  c[1] = (int32_t)n_s;
  c[2] = n_groups;
  c[4] = (int32_t)(uint32_t)(uint64_t)in.bases[0];
  c[5] = (int32_t)(uint32_t)((uint64_t)in.bases[0] >> 32);
  c[6] = in.user_rec;  // user-space record bytes
  c[7] = 64;           // 64-byte spans
  for (int q = 1; q < 4; ++q) {
    c[8 + 2 * (q - 1)] = (int32_t)(uint32_t)(uint64_t)in.bases[q];
    c[9 + 2 * (q - 1)] = (int32_t)(uint32_t)((uint64_t)in.bases[q] >> 32);
  }
  c[15] = (int32_t)n_k;
  int32_t* lab = reinterpret_cast<int32_t*>(head_host_[b] + kHeadBytes);
  for (int g = 0; g < cfg_.group_cap; ++g) lab[g] = (in.labels && g < n_groups) ? in.labels[g] : -1;
  // DMAs once window k - nb (the device block's previous reader) computed: the BPF ring's
  // bytes, the user-space records and the spans, back to back on the copy stream (or over two
  // streams with MISLO_COPY_STREAMS=2); the head is loaded on the compute stream (below).
  HIPCHECK(hipStreamWaitEvent(copy_, compute_done_[b], 0));
  HIPCHECK(hipStreamWaitEvent(copy2_, compute_done_[b], 0));
  HIPCHECK(hipEventRecord(t_start_[b], copy_));
  uint8_t* dst = in_dev_[b];
  size_t st_off = 0;
  auto lap = [](std::chrono::steady_clock::time_point& t, double& acc) {
    const auto n = std::chrono::steady_clock::now();
    acc += std::chrono::duration<double, std::micro>(n - t).count();
    t = n;
  };
  auto tq = std::chrono::steady_clock::now();
  dma(in.kernel, dst + off_kern_, kern_bytes(), staging_[b], st_off, copy_);
  lap(tq, split_us_[0]);
  lap(tq, split_us_[1]);
  dma(in.user, dst + off_user_, 64 * (size_t)cfg_.user_cap, staging_[b], st_off, copy2_);
  lap(tq, split_us_[2]);
  dma(in.spans, dst + off_span_, 64 * (size_t)cfg_.span_cap, staging_[b], st_off, copy2_);
  lap(tq, split_us_[3]);
  HIPCHECK(hipEventRecord(h2d_part_[b], copy2_));
  HIPCHECK(hipEventRecord(h2d_done_[b], copy_));
  HIPCHECK(hipEventRecord(t_copy_end_[b], copy2_));
  const auto te = std::chrono::steady_clock::now();
  dma_us_ += std::chrono::duration<double, std::micro>(te - td).count();
  HIPCHECK(hipStreamWaitEvent(compute_, h2d_done_[b], 0));
  HIPCHECK(hipStreamWaitEvent(compute_, h2d_part_[b], 0));
  HIPCHECK(hipStreamWaitEvent(compute_, comm_done_[b], 0));  // packet b no longer reduced / read
  const bool injected = !inject_.empty();
  if (injected) {
    // rows as the other GPUs would have delivered them (tests, replays): on the device before the
    // window's timed chain (the all-gather they stand for is not the chain's), after window k-1's
    // merge read the receive buffer (compute stream order); the host copy is released here
    HIPCHECK(hipMemcpyAsync(xrecv_, inject_.data(), inject_.size(), hipMemcpyHostToDevice, compute_));
    HIPCHECK(hipStreamSynchronize(compute_));
  }
  HIPCHECK(hipEventRecord(t_comp0_[b], compute_));
  // the head (counts, epoch bases, labels: < 1 KiB) by a kernel load from pinned host memory on
  // the compute stream: a small hipMemcpyAsync H2D is written by the host through the BAR and
  // blocks this thread, and a kernel on the copy stream put ~25 us of queue hand-offs between
  // the window's DMAs (measured); the compute stream has the slack
  to_host(head_host_[b], dst, off_kern_, compute_);
  HIPCHECK(hipEventRecord(head_done_[b], compute_));
  if (cfg_.device_refit && k >= nb_) {
    // fold window k - nb's all-reduced statistics (packet b) and refit before window k: a
    // deterministic prequential lag of nb, identical on every rank
    launch_refit_nb(stats_acc_, packet_dev_[b] + kStatsOff, p0_, cfg_.alpha, cfg_.prior_pseudo, cfg_.n_dom,
                    reinterpret_cast<PosteriorModel*>(model_dev_), compute_, cfg_.inv_temp, cfg_.min_count,
                    p0_ + kSlots * 16, cfg_.cap_dom, cfg_.lik_ceil);
    ++folded_;
  }
  const bool xchg = exchange() || injected;
  const auto tl = std::chrono::steady_clock::now();
  pre_us_ += std::chrono::duration<double, std::micro>(tl - te).count();
  if (!xchg) {
    launch_part(0, b, n_groups, with_labels, learn, false);
  } else {
    if (xspan_) {
      // the window head, then the span side (decode, partition, sort: it reads only the span DMA
      // and the reset accumulators) on side_ while part 1 decodes the records; joined before part 2
      launch_part(4, b, n_groups, with_labels, learn, true);
      HIPCHECK(hipEventRecord(ev_fork_, compute_));
      HIPCHECK(hipStreamWaitEvent(side_, ev_fork_, 0));
      launch_part(3, b, n_groups, with_labels, learn, true);
      HIPCHECK(hipEventRecord(ev_spans_, side_));
    }
    launch_part(1, b, n_groups, with_labels, learn, true);
    // the exchange sits between the window's two halves: every GPU's trace rows of THIS window
    if (injected) {  // rows as the other GPUs would have delivered them (copied above)
      launch_remote_merge(xrecv_, inject_stride_, inject_world_, inject_me_, imp_[b], remote_n_ + b,
                          (uint32_t)cfg_.import_cap, cfg_.xchg_cap, compute_, dbg_ + kDbgXchgDropped);
      inject_.clear();
      launch_window_rows(reinterpret_cast<const int*>(in_dev_[b]), remote_n_ + b, n_rows_, rows_, gen_, compute_);
    } else if (xcomm_) {
      // on the compute stream, over the exchange's own communicator (each communicator is used
      // on one stream only, so each keeps one issue order on every rank): part 2 follows the
      // merge in stream order, with no hand-off between hardware queues on the window's critical
      // path (each such hop idled the compute queue 20-45 us, profiles/r5_multigpu/)
      NCCLCHECK(ncclAllGather(xsend_, xrecv_, xstride_, ncclUint8, xcomm_, compute_));
      launch_remote_merge(xrecv_, xstride_, world_, rank_, imp_[b], remote_n_ + b, (uint32_t)cfg_.import_cap,
                          cfg_.xchg_cap, compute_, dbg_ + kDbgXchgDropped);
      launch_window_rows(reinterpret_cast<const int*>(in_dev_[b]), remote_n_ + b, n_rows_, rows_, gen_, compute_);
    } else {
      // MISLO_XCHG_STREAM=comm: the exchange on the comm stream with the window's other
      // collectives: the compute stream hands over after part 1 and waits for the merge
      HIPCHECK(hipEventRecord(xchg_done_[b], compute_));
      HIPCHECK(hipStreamWaitEvent(comm_stream_, xchg_done_[b], 0));
      NCCLCHECK(ncclAllGather(xsend_, xrecv_, xstride_, ncclUint8, comm_, comm_stream_));
      launch_remote_merge(xrecv_, xstride_, world_, rank_, imp_[b], remote_n_ + b, (uint32_t)cfg_.import_cap,
                          cfg_.xchg_cap, comm_stream_, dbg_ + kDbgXchgDropped);
      launch_window_rows(reinterpret_cast<const int*>(in_dev_[b]), remote_n_ + b, n_rows_, rows_, gen_, comm_stream_);
      HIPCHECK(hipEventRecord(xchg_done_[b], comm_stream_));
      HIPCHECK(hipStreamWaitEvent(compute_, xchg_done_[b], 0));
    }
    if (xspan_) HIPCHECK(hipStreamWaitEvent(compute_, ev_spans_, 0));
    launch_part(2, b, n_groups, with_labels, learn, true);
  }
  const auto tt = std::chrono::steady_clock::now();
  launch_us_ += std::chrono::duration<double, std::micro>(tt - tl).count();
  // per-incident results of this window (the buffers are reused by the next window); one GPU:
  // copied by the graph's k_window_end
  if (comm_) to_host(res_dev_[b], res_host_[b], res_bytes_, compute_);
  HIPCHECK(hipEventRecord(t_comp1_[b], compute_));
  HIPCHECK(hipEventRecord(compute_done_[b], compute_));
  HIPCHECK(hipStreamWaitEvent(comm_stream_, compute_done_[b], 0));
  if (comm_) {
    // one group: the node-wide packet and the node-wide incident list. The ring accounting at
    // the packet's tail stays this GPU's own (each GPU is a consumer of its rings: its first busy
    // record, its records), so it is left out of the sum.
    NCCLCHECK(ncclGroupStart());
    NCCLCHECK(ncclAllReduce(packet_dev_[b], packet_dev_[b], kPacketLen - kPacketRing, ncclFloat64, ncclSum, comm_,
                            comm_stream_));
    NCCLCHECK(ncclAllGather(res_dev_[b], res_all_dev_[b], res_bytes_, ncclUint8, comm_, comm_stream_));
    NCCLCHECK(ncclGroupEnd());
    to_host(res_all_dev_[b], res_all_host_[b], res_bytes_ * world_, comm_stream_);
  }
  if (comm_)
    hipLaunchKernelGGL(k_accumulate, dim3((kPacketLen + 255) / 256), dim3(256), 0, comm_stream_, packet_dev_[b],
                       totals_, kPacketLen, packet_host_[b]);
  HIPCHECK(hipEventRecord(t_end_[b], comm_stream_));
  HIPCHECK(hipEventRecord(comm_done_[b], comm_stream_));
  ++submitted_;
  const auto t1 = std::chrono::steady_clock::now();
  tail_us_ += std::chrono::duration<double, std::micro>(t1 - tt).count();
  issue_us_ += std::chrono::duration<double, std::micro>(t1 - t0).count();
  ++issue_n_;
}

bool WindowEngine::query(int64_t k) {
  const hipError_t e = hipEventQuery(comm_done_[k % nb_]);
  if (e == hipSuccess) return true;
  if (e == hipErrorNotReady) return false;
  HIPCHECK(e);
  return false;
}

void WindowEngine::wait(int64_t k) {
  if (spin_) {  // poll: no interrupt wake-up latency (flat-out benchmarking; costs a core)
    for (;;) {
      const hipError_t e = hipEventQuery(comm_done_[k % nb_]);
      if (e == hipSuccess) return;
      if (e != hipErrorNotReady) HIPCHECK(e);
    }
  }
  HIPCHECK(hipEventSynchronize(comm_done_[k % nb_]));
}

ResultView WindowEngine::results(int64_t k) const {
  const uint8_t* r = res_host_[k % nb_];
  const size_t G = cfg_.group_cap;
  const size_t o_gconf = 16 * G * 8, o_feat = o_gconf + G * 8, o_pred = o_feat + 16 * G * 4, o_ev = o_pred + G * 4;
  const size_t o_sli = o_ev + 16 * G * 4;
  return ResultView{reinterpret_cast<const double*>(r), reinterpret_cast<const double*>(r + o_gconf),
                    reinterpret_cast<const float*>(r + o_feat), reinterpret_cast<const int32_t*>(r + o_pred),
                    reinterpret_cast<const uint32_t*>(r + o_ev), reinterpret_cast<const uint32_t*>(r + o_sli),
                    reinterpret_cast<const uint32_t*>(r + o_sli) + 2 * G,
                    reinterpret_cast<const uint32_t*>(r + o_sli) + 4 * G};
}

std::vector<float> WindowEngine::copy_ms(int64_t k) {
  // [copy duration of window k, copy-engine idle time between window k-1's DMAs and k's]
  const int b = (int)(k % nb_);
  float dur = 0.f, gap = -1.f;
  HIPCHECK(hipEventSynchronize(t_copy_end_[b]));
  HIPCHECK(hipEventElapsedTime(&dur, t_start_[b], t_copy_end_[b]));
  if (k >= 1 && nb_ > 1) HIPCHECK(hipEventElapsedTime(&gap, t_copy_end_[(k - 1) % nb_], t_start_[b]));
  return {dur, gap};
}

std::pair<float, float> WindowEngine::window_ms(int64_t k) {
  const int b = (int)(k % nb_);
  float total = 0.f, comp = 0.f;
  HIPCHECK(hipEventSynchronize(t_end_[b]));
  HIPCHECK(hipEventElapsedTime(&total, t_start_[b], t_end_[b]));
  HIPCHECK(hipEventElapsedTime(&comp, t_comp0_[b], t_comp1_[b]));
  return {total, comp};
}

void WindowEngine::set_model_bytes(const void* bytes, size_t n) {
  if (n != sizeof(PosteriorModel)) throw std::invalid_argument("model image must be POSTERIOR_MODEL_BYTES bytes");
  // a pinned staging slot not read by any queued copy: at most max_ahead windows are queued
  uint8_t* h = model_host_[model_slot_++ % model_host_.size()];
  std::memcpy(h, bytes, n);
  HIPCHECK(hipMemcpyAsync(model_dev_, h, n, hipMemcpyHostToDevice, compute_));
}

void WindowEngine::set_app_model(const void* bytes, size_t n) {
  if (n != sizeof(AppModel)) throw std::invalid_argument("application model must be APP_MODEL_BYTES bytes");
  uint8_t* h = model_host_[model_slot_++ % model_host_.size()];  // pinned slots hold a PosteriorModel
  static_assert(sizeof(AppModel) <= sizeof(PosteriorModel), "the staging slots fit the application model");
  std::memcpy(h, bytes, n);
  HIPCHECK(hipMemcpyAsync(app_dev_, h, n, hipMemcpyHostToDevice, compute_));
}

void WindowEngine::set_p0(const double* p0, size_t n) {
  if (n != (size_t)kSlots * 16 && n != 2 * (size_t)kSlots * 16) throw std::invalid_argument("p0 must be f64[256] or [512]");
  HIPCHECK(hipMemset(p0_ + kSlots * 16, 0, kSlots * 16 * sizeof(double)));  // [256]: no floor
  HIPCHECK(hipMemcpy(p0_, p0, n * sizeof(double), hipMemcpyHostToDevice));
}

void WindowEngine::set_refit(double alpha, double prior_pseudo, double inv_temp, double min_count, int cap_dom,
                             double ceil) {
  if (!(alpha > 0.0) || !(prior_pseudo >= 0.0) || !(inv_temp > 0.0) || !(min_count >= 0.0) || cap_dom >= cfg_.n_dom ||
      !(ceil > 0.0 && ceil <= 1.0))
    throw std::invalid_argument("refit parameters");
  cfg_.lik_ceil = ceil;
  cfg_.cap_dom = cap_dom < 0 ? -1 : cap_dom;
  cfg_.alpha = alpha;
  cfg_.prior_pseudo = prior_pseudo;
  cfg_.inv_temp = inv_temp;
  cfg_.min_count = min_count;
}

void WindowEngine::refit_now() {
  launch_refit_nb(stats_acc_, nullptr, p0_, cfg_.alpha, cfg_.prior_pseudo, cfg_.n_dom,
                  reinterpret_cast<PosteriorModel*>(model_dev_), compute_, cfg_.inv_temp, cfg_.min_count,
                    p0_ + kSlots * 16, cfg_.cap_dom, cfg_.lik_ceil);
}

void WindowEngine::score_features(const float* feat, int n, const int32_t* labels, double* post, int32_t* pred,
                                  double* conf, uint32_t* evbits, uint32_t* confusion, const uint32_t* app_cnt) {
  if (n < 0) throw std::invalid_argument("n");
  sync();
  if (n == 0) return;
  // one scratch block: [n][16] f32 features | n | labels | post | pred | conf | evbits | confusion |
  // application counts [n][2]
  const size_t o_n = (size_t)n * 16 * 4, o_lab = o_n + 64, o_post = (o_lab + (size_t)n * 4 + 63) & ~size_t(63);
  const size_t o_pred = o_post + (size_t)n * 16 * 8, o_conf = (o_pred + (size_t)n * 4 + 63) & ~size_t(63);
  const size_t o_ev = o_conf + (size_t)n * 8, o_cm = o_ev + (size_t)n * 16 * 4, o_app = o_cm + 16 * 16 * 4;
  const size_t bytes = o_app + (size_t)n * 2 * 4;
  uint8_t* d = dalloc<uint8_t>(bytes);
  HIPCHECK(hipMemset(d, 0, bytes));
  HIPCHECK(hipMemcpy(d, feat, o_n, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(d + o_n, &n, sizeof(int), hipMemcpyHostToDevice));
  if (labels) HIPCHECK(hipMemcpy(d + o_lab, labels, (size_t)n * 4, hipMemcpyHostToDevice));
  if (app_cnt) HIPCHECK(hipMemcpy(d + o_app, app_cnt, (size_t)n * 2 * 4, hipMemcpyHostToDevice));
  launch_posterior(reinterpret_cast<const float*>(d), reinterpret_cast<const int*>(d + o_n), n,
                   reinterpret_cast<const PosteriorModel*>(model_dev_),
                   labels ? reinterpret_cast<const int32_t*>(d + o_lab) : nullptr, reinterpret_cast<double*>(d + o_post),
                   reinterpret_cast<int32_t*>(d + o_pred), reinterpret_cast<double*>(d + o_conf),
                   reinterpret_cast<uint32_t*>(d + o_ev), reinterpret_cast<uint32_t*>(d + o_cm), compute_,
                   app_cnt ? app_dev_ : nullptr, app_cnt ? reinterpret_cast<const uint32_t*>(d + o_app) : nullptr);
  HIPCHECK(hipStreamSynchronize(compute_));
  HIPCHECK(hipMemcpy(post, d + o_post, (size_t)n * 16 * 8, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(pred, d + o_pred, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(conf, d + o_conf, (size_t)n * 8, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(evbits, d + o_ev, (size_t)n * 16 * 4, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(confusion, d + o_cm, 16 * 16 * 4, hipMemcpyDeviceToHost));
  HIPCHECK(hipFree(d));
}

void WindowEngine::set_pods(const uint32_t* pods, const uint32_t* svcnode, size_t n) {
  // the host mirror is only written between the previous upload's completion (compute stream
  // order: the upload precedes later windows) and this call; uploads are rare (pod churn)
  HIPCHECK(hipStreamSynchronize(compute_));
  for (size_t i = 0; i < n; ++i)
    if (pods[i] < kPodRows) pod_host_[pods[i]] = svcnode[i];
  HIPCHECK(hipMemcpyAsync(pod_sn_, pod_host_, kPodRows * 4, hipMemcpyHostToDevice, compute_));
}

std::vector<uint8_t> WindowEngine::sent_block() {
  sync();
  std::vector<uint8_t> out(xsend_ ? xstride_ : 0);
  if (xsend_) HIPCHECK(hipMemcpy(out.data(), xsend_, xstride_, hipMemcpyDeviceToHost));
  return out;
}

std::vector<int64_t> WindowEngine::import_state() {
  sync();
  int rows[2];
  unsigned long long tmax = 0;
  GenMeta g{};
  std::vector<uint32_t> r(nb_);
  HIPCHECK(hipMemcpy(rows, rows_, sizeof(rows), hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(&tmax, tmax_, 8, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(&g, gen_, sizeof(g), hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(r.data(), remote_n_, 4 * nb_, hipMemcpyDeviceToHost));
  // rows[0..1], tmax, generations, current slot, windows held, per age: cut-off and rows, per
  // buffer: other GPUs' rows
  std::vector<int64_t> out{rows[0], rows[1], (int64_t)tmax, gens_, g.cur, g.filled};
  for (int a = 0; a < kMaxGens; ++a) out.push_back(g.cut[a]);
  for (int a = 0; a < kMaxGens; ++a) out.push_back(a < gens_ ? g.n_rows[(g.cur + gens_ - a) % gens_] : 0);
  for (int b = 0; b < nb_; ++b) out.push_back(r[b]);
  return out;
}

void WindowEngine::inject_remote(const void* blocks, size_t stride, int world, int me) {
  if (!cfg_.import_cap || !cfg_.xchg_cap) throw std::logic_error("inject_remote needs import_cap and xchg_cap > 0");
  if (world < 1 || me < 0 || me >= world || stride < sizeof(XRec)) throw std::invalid_argument("bad exchange blocks");
  const uint8_t* h = static_cast<const uint8_t*>(blocks);
  for (int r = 0; r < world; ++r) {  // the merge kernel trusts each block's header: check it here
    uint32_t c;
    std::memcpy(&c, h + (size_t)r * stride, 4);
    if ((size_t)c * sizeof(XRec) + sizeof(XRec) > stride) throw std::invalid_argument("block row count exceeds stride");
    if (r != me && c > (uint32_t)cfg_.xchg_cap) throw std::invalid_argument("block holds more rows than xchg_cap");
  }
  if (stride * world > xrecv_bytes_) {
    sync();
    if (xrecv_) HIPCHECK(hipFree(xrecv_));
    xrecv_ = dalloc<uint8_t>(stride * world);
    xrecv_bytes_ = stride * world;
  }
  inject_.assign(h, h + stride * world);  // consumed by the next submit, between its two halves
  inject_stride_ = stride;
  inject_world_ = world;
  inject_me_ = me;
}

void WindowEngine::init_comm(const ncclUniqueId& id, int rank, int world) {
  if (comm_) throw std::logic_error("communicator already initialised");
  // world 1 is a real communicator too: every collective of the window chain runs (on one rank),
  // which is how a one-GPU box exercises the multi-GPU path (tests/test_rccl_single.py)
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("communicator rank / world");
  if (submitted_) throw std::logic_error("init_comm before the first window");
  HIPCHECK(hipSetDevice(cfg_.device));
  NCCLCHECK(ncclCommInitRank(&comm_, world, id, rank));
  {
    // the comm stream at its own priority: streams of one priority share that priority's
    // hardware queues (GPU_MAX_HW_QUEUES, 4 by default), and a comm stream landing on the copy
    // stream's queue held window k+1's DMAs behind window k's collectives -- which wait for window
    // k's compute -- so no two windows overlapped (measured with a one-rank communicator,
    // tools/rccl_overlap.py: copy-engine idle 0.65-0.75 ms per window, 1.27-1.35 ms per window
    // against 0.77 ms without a communicator). MISLO_COMM_STREAM_PRIO=0: the default priority.
    int lo = 0, hi = 0;
    HIPCHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    const char* pv = getenv("MISLO_COMM_STREAM_PRIO");
    if (pv && atoi(pv) == 0)
      HIPCHECK(hipStreamCreateWithFlags(&comm_stream_, hipStreamNonBlocking));
    else
      HIPCHECK(hipStreamCreateWithPriority(&comm_stream_, hipStreamNonBlocking, hi));
  }
  rank_ = rank;
  world_ = world;
  for (int b = 0; b < nb_; ++b) {
    res_all_dev_.push_back(dalloc<uint8_t>(res_bytes_ * world));
    res_all_host_.push_back(static_cast<uint8_t*>(host_block(res_bytes_ * world)));
  }
  if (cfg_.xchg_cap) {
    if (world > 8) throw std::invalid_argument("the exchange is sized for <= 8 GPUs per node");
    if (xrecv_) HIPCHECK(hipFree(xrecv_));
    xrecv_ = dalloc<uint8_t>(xstride_ * world);
    xrecv_bytes_ = xstride_ * world;
    HIPCHECK(hipMemset(xrecv_, 0, xrecv_bytes_));
    // The exchange runs on the comm stream with the window's other collectives: one communicator,
    // one stream, one issue order on every rank. MISLO_XCHG_STREAM=compute puts it on the compute
    // stream over a communicator of its own (ncclCommSplit: 0.60 against 0.62 ms per window in the
    // one-rank rehearsal, profiles/r5_multigpu/); two communicators then run collectives on two
    // streams at once, which no run with world >= 2 has exercised yet, so it is opt-in. Rank 0's
    // choice is broadcast first: ncclCommSplit is collective, and ranks with another env must
    // neither hang in it nor skip it.
    const char* xv = getenv("MISLO_XCHG_STREAM");
    int split = (xv && std::strcmp(xv, "compute") == 0) ? 1 : 0;
    int* d_split = dalloc<int>(1);
    HIPCHECK(hipMemcpy(d_split, &split, sizeof(int), hipMemcpyHostToDevice));
    NCCLCHECK(ncclBroadcast(d_split, d_split, 1, ncclInt32, 0, comm_, comm_stream_));
    HIPCHECK(hipStreamSynchronize(comm_stream_));
    HIPCHECK(hipMemcpy(&split, d_split, sizeof(int), hipMemcpyDeviceToHost));
    HIPCHECK(hipFree(d_split));
    if (split) NCCLCHECK(ncclCommSplit(comm_, 0, rank, &xcomm_, nullptr));
  }
}

void WindowEngine::totals(double* out) {
  sync();
  HIPCHECK(hipMemcpy(out, totals_, kPacketLen * sizeof(double), hipMemcpyDeviceToHost));
}

void WindowEngine::reset_totals() {
  sync();
  HIPCHECK(hipMemset(totals_, 0, kPacketLen * sizeof(double)));
}

void WindowEngine::stats_acc(double* out) {
  sync();
  HIPCHECK(hipMemcpy(out, stats_acc_, kStatsLen * sizeof(double), hipMemcpyDeviceToHost));
}

void WindowEngine::restore(const double* stats, const void* model, size_t n, int64_t folded) {
  if (n && n != sizeof(PosteriorModel)) throw std::invalid_argument("model image must be POSTERIOR_MODEL_BYTES bytes");
  sync();
  HIPCHECK(hipMemcpy(stats_acc_, stats, kStatsLen * sizeof(double), hipMemcpyHostToDevice));
  if (n) {
    HIPCHECK(hipMemcpy(model_dev_, model, n, hipMemcpyHostToDevice));
  } else {  // the learned model from the restored statistics, by the device refit itself
    launch_refit_nb(stats_acc_, nullptr, p0_, cfg_.alpha, cfg_.prior_pseudo, cfg_.n_dom,
                    reinterpret_cast<PosteriorModel*>(model_dev_), compute_, cfg_.inv_temp, cfg_.min_count,
                    p0_ + kSlots * 16, cfg_.cap_dom, cfg_.lik_ceil);
    HIPCHECK(hipStreamSynchronize(compute_));
  }
  folded_ = folded;
}

void WindowEngine::model_bytes(void* out) {
  sync();
  HIPCHECK(hipMemcpy(out, model_dev_, sizeof(PosteriorModel), hipMemcpyDeviceToHost));
}

void WindowEngine::sync() {
  HIPCHECK(hipStreamSynchronize(copy_));
  if (copy2_ != copy_) HIPCHECK(hipStreamSynchronize(copy2_));
  HIPCHECK(hipStreamSynchronize(compute_));
  HIPCHECK(hipStreamSynchronize(comm_stream_));
}

}  // namespace mislo
