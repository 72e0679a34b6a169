// kb_capi.hip -- host side of the C-ABI (include/kalibr_hip.h): buffer management, launch
// sequencing, the hipGraph-captured device-resident optimizer loop and the RCCL exchange.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/kalibr_hip.h"
#include "kb_kernels.hip"
#include "kb_pcg.hip"

using namespace kb;

namespace {
thread_local std::string g_err;

int fail(const std::string& m) {
  g_err = m;
  return -1;
}

#define KB_HIP(call)                                                                              \
  do {                                                                                            \
    hipError_t e_ = (call);                                                                       \
    if (e_ != hipSuccess) return fail(std::string(#call) + ": " + hipGetErrorString(e_));        \
  } while (0)

#define KB_NCCL(call)                                                                             \
  do {                                                                                            \
    ncclResult_t r_ = (call);                                                                     \
    if (r_ != ncclSuccess) return fail(std::string(#call) + ": " + ncclGetErrorString(r_));      \
  } while (0)

int nintr_host(int m) {
  switch (m) {
    case KB_PINHOLE_RADTAN: return 8;
    case KB_OMNI_RADTAN: return 9;
    case KB_EUCM: return 6;
    case KB_OMNI: return 5;
    case KB_DS: return 6;
    case KB_PINHOLE_EQUI: return 8;
    case KB_PINHOLE_FOV: return 5;
    default: return -1;
  }
}
}  // namespace

constexpr int kGraphPasses = 8;  // optimizer passes per captured multi-pass graph
constexpr int kGnOneGraph = 64;  // kb_gn_launch: runs of up to this many GN passes are one graph (with the loop's end)
constexpr int kXMaxRanks = 64;
constexpr int kPolicyMarginal = 2;  // graph policy id of kb_optimize_marginal's passes (GN over the marginal solve)   // expanded partials: per-rank max|dx_f| slots in the image's aux area
constexpr int kLocalMaxRanks = 16;  // kb_comm_init_local group size

// In-process group of sharded handles (kb_comm_init_local): the collectives become device copies between the
// members' buffers, ordered by HIP events and a host barrier (one host thread per member).
struct kb_local_group {
  int n = 0;
  int refs = 0;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  long gen = 0;
  bool broken = false;  // a member timed out: every later barrier fails at once
  std::vector<hipEvent_t> ready, done;
  std::vector<const double*> src;
  // false on timeout (a member never arrived)
  bool barrier() {
    std::unique_lock<std::mutex> lk(m);
    if (broken) return false;
    const long g = gen;
    if (++arrived == n) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return true;
    }
    if (!cv.wait_for(lk, std::chrono::seconds(60), [&] { return gen != g || broken; }) || broken) {
      broken = true;
      cv.notify_all();
      return false;
    }
    return true;
  }
};

struct LocalSrc {
  const double* p[kLocalMaxRanks];
};

// out[i] = sum_r src_r[i] in rank order (sum) or out[r * count + i] = src_r[i] (gather)
__global__ void __launch_bounds__(256) k_local_coll(LocalSrc s, int n, size_t count, double* out, int gather) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
    if (gather) {
      for (int r = 0; r < n; ++r) out[(size_t)r * count + i] = s.p[r][i];
    } else {
      double a = s.p[0][i];
      for (int r = 1; r < n; ++r) a += s.p[r][i];
      out[i] = a;
    }
  }
}

struct kb_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  KbDev d{};
  int N = 0, F = 0, K = 0, V = 0, NC = 0, C = 0, ncols = 0, S = 0, W = 0;
  int WPB = 1;
  bool build_pipe = false;  // k_buildp (one wave per camera, N + 2 waves) instead of k_build
  bool xexp = false;        // GN fused passes with expanded partials (C > 64, k_buildp): k_colsumx, no k_colimg
  std::vector<int32_t> vcam;  // camera of each view (host copy: the algorithmic flop count)
  // growth in place (kb_append_frames / kb_drop_last_frames): device capacities and host mirrors of the view layout
  int bpc = 1;                      // k_buildp blocks per CU (frames per block = ceil(F / (256 bpc)))
  int F_cap = 0, V_cap = 0, NC_cap = 0;
  int part_rows = 0;                // rows of d.part (build blocks it holds): nblk(F) is not monotone in F
  std::vector<uint32_t> vo_host;    // [V + 1] view offsets
  std::vector<int32_t> frame_v0;    // [F + 1] first view of each frame (frame_v0[F] = V)
  size_t pcg_F = 0, rjr_F = 0, cond_n = 0;  // frame count / columns the lazily allocated buffers are sized for
  double* ximg_part = nullptr;  // sharded + xexp: this rank's partial image (all-reduced into d.simg)
  std::vector<void*> xar_opened;  // peers' exchange regions mapped by IPC handles (closed by kb_destroy)
  bool xar_failed = false;        // a k_xar wait of this rank timed out (comm_check): agreed on at the next loop start
  double* xar_agree_buf = nullptr;  // [2]: this rank's failure flag | the sum over the ranks
  bool buildp_wide = false;  // k_buildp<.., MW = 8> (multi-model rigs with <= 8 waves per block)
  double* rjr = nullptr;     // [F + 1] kb_rhs_jtj_rhs: per-frame terms | result
  int gn_prepared = -1;      // kb_gn_prepare'd pass count, consumed by kb_gn_launch (-1: nothing prepared; every
                             // entry point that changes the state, the graphs or the control block resets it)
  bool sys_valid = false;    // the per-call system of the last kb_build is intact (H_ff, H_fc, g_f, H_cc, g_c): the
                             // device-resident loops overwrite g_c and skip the frame-block stores in GN fused passes
  size_t lds_colimg = 0;     // k_colimg's staging (per-camera sums, chains, T, column info)
  bool gn_graph = false;
  int build_threads = 64;
  size_t lds_build = 0, lds_camexp = 0, lds_schur = 0, lds_solve = 0;
  int solve_threads = 64;
  int mb = 7, ms = 7;  // Schur-sum tiles per wave of k_build / k_schur (template bucket)
  const void* fn_build = nullptr;
  const void* fn_build_gn = nullptr;  // GN fused passes
  const void* fn_schur = nullptr;
  const void* fn_solve = nullptr;
  int cur = 0;  // host mirror of ctrl->cur for the per-call path
  bool uploaded = false;
  std::vector<void*> allocs;
  // loop
  // graphs[k]: k captured passes of graph_policy back to back (no inter-launch gap between them), k = 1..kGraphPasses;
  // a run of n passes launches n / kGraphPasses full graphs and one graph of the remainder (captured on first use)
  hipGraphExec_t graphs[kGraphPasses + 1] = {};
  int graph_policy = -1;
  // kb_gn_prepare / kb_gn_launch: the last gn_tail_n GN passes and the loop's end (the last step's back-substitution
  // and k_post) in one graph, after gn_head passes of whole kGraphPasses graphs
  hipGraphExec_t gn_tail = nullptr, gn_big = nullptr;  // gn_big: kGnOneGraph passes (the head of longer runs)
  int gn_tail_n = -1, gn_head = 0;
  bool graph_failed = false;  // capture of the RCCL calls failed once: eager passes from then on
  int graph_trace_cap = 0;
  double* trace = nullptr;
  int trace_cap = 0;
  // sharding
  ncclComm_t comm = nullptr;
  kb_local_group* lg = nullptr;  // in-process group (kb_comm_init_local) instead of RCCL
  int nranks = 1, rank = 0;
  double* psum_red = nullptr;   // [Wtot] all-reduced finished column sums (sharded, per-call path)
  double* psum_red8 = nullptr;  // [8][Wtot] all-reduced stage-1 rows (sharded optimizer loop)
  double* bpart_all = nullptr;  // [nranks][F_max][4] all-gathered per-frame step rows (sharded)
  bool gn_fuse = true;          // GN passes fused (KB_GN_FUSED=0: the general pass, for comparison)
  int F_max = 0;
  // build-kernel timing
  double build_ms = 0.0;
  double* marg_buf = nullptr;  // marginal solver outputs, solve then analyze: V [C][C] | sv [C] | info [8]
  KbMarg marg{};               // kb_optimize_marginal: the k_marg arguments its captured passes use
  size_t lds_marg = 0;
  // linear solver of kb_solve: KB_SOLVER_SCHUR (direct) or KB_SOLVER_PCG (LinearSolverPCG)
  int solver_kind = KB_SOLVER_SCHUR;
  kb_pcg_options pcg{1e-6, -1, 1};
  double pcg_residual = -1.0;  // LinearSolverPCG::_residual (init(): -1)
  kb_pcg_info pcg_info{0, 0.0, 0.0};
  double* cond2 = nullptr;     // setConditioner: squared diagonal [ncols] (canonical order)
  bool use_cond = false;       // kb_set_conditioner active (kb_set_constant_conditioner clears it)
  double* pcg_buf = nullptr;   // part [F][C+1] | part2 [F] | info [8] | PCG_SCHUR info [4]
  int* pcg_cb = nullptr;       // [2][C] camera DV block start / size per column
  unsigned* pcg_bar = nullptr;

  template <class T>
  int alloc(T** p, size_t n) {
    void* q = nullptr;
    if (n == 0) n = 1;
    hipError_t e = hipMalloc(&q, n * sizeof(T));
    if (e != hipSuccess) return fail(std::string("hipMalloc: ") + hipGetErrorString(e));
    hipMemsetAsync(q, 0, n * sizeof(T), stream);
    allocs.push_back(q);
    *p = (T*)q;
    return 0;
  }
};

// The build kernels of each camera-model set live in their own translation unit (kb_build_tu.hip, -DKB_TU_ID=id):
// kb_build_fn_<id>(gn, mb, pipe, wide) returns the k_build / k_buildp instantiation (mb: Schur tiles per wave of
// k_build 1 | 4 | 7, or per frame wave of k_buildp 5 | 7).
#define KB_BUILD_TU_DECL(id) const void* kb_build_fn_##id(bool gn, int mb, bool pipe, bool wide);
KB_BUILD_TU_DECL(0)
KB_BUILD_TU_DECL(1)
KB_BUILD_TU_DECL(2)
KB_BUILD_TU_DECL(3)
KB_BUILD_TU_DECL(4)
KB_BUILD_TU_DECL(5)
KB_BUILD_TU_DECL(6)
KB_BUILD_TU_DECL(7)
KB_BUILD_TU_DECL(8)

// Build kernel for the rig's camera-model set `mm` (bit m = model m present).
template <bool GN>
static const void* pick_build(int mb, unsigned mm, bool pipe, bool wide) {
  switch (mm) {
    case 1u << KB_PINHOLE_RADTAN: return kb_build_fn_0(GN, mb, pipe, wide);
    case 1u << KB_OMNI_RADTAN: return kb_build_fn_1(GN, mb, pipe, wide);
    case 1u << KB_EUCM: return kb_build_fn_2(GN, mb, pipe, wide);
    case 1u << KB_OMNI: return kb_build_fn_3(GN, mb, pipe, wide);
    case 1u << KB_DS: return kb_build_fn_4(GN, mb, pipe, wide);
    case 1u << KB_PINHOLE_EQUI: return kb_build_fn_5(GN, mb, pipe, wide);
    case 1u << KB_PINHOLE_FOV: return kb_build_fn_6(GN, mb, pipe, wide);
    case (1u << KB_OMNI_RADTAN) | (1u << KB_EUCM): return kb_build_fn_7(GN, mb, pipe, wide);
    default: return kb_build_fn_8(GN, mb, pipe, wide);
  }
}

// frames per build block for F frames
static int gframes_for(const kb_handle* h, int F) {
  return h->build_pipe ? (F + 256 * h->bpc - 1) / (256 * h->bpc) : (F + 511) / 512;
}

// the frame-count-dependent layout: columns, state size, build blocks (frames per block), step rows
static void set_frame_counts(kb_handle* h) {
  KbDev& d = h->d;
  h->ncols = h->C + 6 * h->F;
  h->S = h->N * KB_MAX_INTR + 7 * (h->N - 1) + 7 * h->F;
  d.F = h->F;
  d.ncols = h->ncols;
  if (d.S < h->S) d.S = h->S;  // d.S: the slot stride of the [2][S] state buffer (its capacity), >= the state size
  d.gframes = gframes_for(h, h->F);
  d.nblk = (h->F + d.gframes - 1) / d.gframes;
  d.nblk_bs = h->F;  // k_backsub: one step row per frame (one wave per frame)
}

// dynamic LDS of the build kernel at `gframes` frames per block (the staged frame poses); *tg: the target corners
// are staged in LDS too.  k_buildp's static LDS (control copies, chain / intrinsic table, column info, counters) is
// below this
constexpr size_t kBuildpStaticLds = 4096;
static size_t build_lds_for(const kb_handle* h, int gframes, int* tg_out) {
  const int N = h->N, C = h->C, WPB = h->d.wpb;
  const int CZ = 16 * ((C + 16) / 16);  // [Y | z] row stride of the Schur tiles
  const int tgl = (3 * h->K <= kTargetLds ? 3 * h->K : 0) + 8 * gframes;
  if (h->build_pipe) {  // k_buildp: tiles | H | chains G | view outputs | frame sums | frame-wave buffers | K | target,
                        // poses | the second view-output buffer
    const int np = N * (N - 1) / 2;
    const size_t vbs = 44 * N + 6 * CZ;  // view outputs dH | dg | intrinsic columns (+ the frame sums in place)
    const size_t base = N * 64 * XS + N * 256 + N * 36 + 2 * vbs + 40 + 6 * CZ + 36 * np + 8 * gframes;
    // the target corners are staged when they fit beside the rest
    const bool tg = 3 * h->K <= kTargetLds && sizeof(double) * (base + 3 * h->K) + kBuildpStaticLds <= 160 * 1024;
    if (tg_out) *tg_out = tg ? 1 : 0;
    return sizeof(double) * (base + (tg ? 3 * h->K : 0));
  }
  if (tg_out) *tg_out = 0;
  return sizeof(double) * (WPB * 64 * XS + WPB * 256 + N * (256 + 256 + 64 + 36 + 36 + 8) + 36 + 16 * CZ +
                           18 * N * (N - 1) + tgl);
}

static size_t build_lds(kb_handle* h) { return build_lds_for(h, h->d.gframes, &h->d.bp_tg); }

// the build kernel's LDS fits at F frames (checked before kb_append_frames / kb_drop_last_frames change anything)
static bool build_lds_fits(const kb_handle* h, int F) {
  return build_lds_for(h, gframes_for(h, F), nullptr) + (h->build_pipe ? kBuildpStaticLds : 0) <= 160 * 1024;
}

static void drop_graphs(kb_handle* h) {
  for (auto& g : h->graphs) {
    if (g) hipGraphExecDestroy(g);
    g = nullptr;
  }
  if (h->gn_tail) hipGraphExecDestroy(h->gn_tail);
  if (h->gn_big) hipGraphExecDestroy(h->gn_big);
  h->gn_tail = h->gn_big = nullptr;
  h->gn_tail_n = -1;
  h->graph_policy = -1;
  h->gn_prepared = -1;  // a prepared GN launch used these graphs
}

// anything that changes the state, the control block or the system behind a kb_gn_prepare'd loop start voids it:
// kb_gn_launch then fails instead of timing passes from a stale prelude
static void unprepare(kb_handle* h) { h->gn_prepared = -1; }

static bool sharded(const kb_handle* h) { return h->comm || h->lg; }

// a k_xar wait that timed out (a peer rank never published its partial image): the pass results are void
static int comm_check(kb_handle* h, const KbCtrl& c) {
  if (!c.comm_err) return 0;
  h->xar_failed = true;  // the next loop start agrees with the other ranks on leaving the direct path
  return fail("direct all-reduce (k_xar): a peer rank did not arrive within the wait bound (KB_XAR_TIMEOUT_MS); the "
              "handle switches to the RCCL collective at its next loop start");
}

// one collective of the in-process group: every member publishes its send buffer and an event, waits for all
// members' events, copies / sums on its own stream, then waits until every member has read its buffer
static int local_coll(kb_handle* h, const double* send, double* recv, size_t count, bool gather) {
  kb_local_group* G = h->lg;
  const int r = h->rank;
  if (send == recv) return fail("kb_comm_init_local: in-place collective");
  G->src[r] = send;
  KB_HIP(hipEventRecord(G->ready[r], h->stream));
  if (!G->barrier()) return fail("kb_comm_init_local: a member of the group did not reach the collective (60 s)");
  LocalSrc ls{};
  for (int j = 0; j < G->n; ++j) {
    KB_HIP(hipStreamWaitEvent(h->stream, G->ready[j], 0));
    ls.p[j] = G->src[j];
  }
  const int blocks = (int)std::min<size_t>((count + 255) / 256, 1024);
  hipLaunchKernelGGL(k_local_coll, dim3(std::max(blocks, 1)), dim3(256), 0, h->stream, ls, G->n, count, recv,
                     gather ? 1 : 0);
  KB_HIP(hipGetLastError());
  KB_HIP(hipEventRecord(G->done[r], h->stream));
  if (!G->barrier()) return fail("kb_comm_init_local: a member of the group did not reach the collective (60 s)");
  for (int j = 0; j < G->n; ++j) KB_HIP(hipStreamWaitEvent(h->stream, G->done[j], 0));
  // nobody re-records ready / done (next collective) before every member has enqueued its waits on them
  if (!G->barrier()) return fail("kb_comm_init_local: a member of the group did not reach the collective (60 s)");
  return 0;
}

// sum over ranks (RCCL or the in-process group); all ranks receive identical bits
static int coll_allreduce(kb_handle* h, const double* send, double* recv, size_t count) {
  if (h->lg) return local_coll(h, send, recv, count, false);
  KB_NCCL(ncclAllReduce(send, recv, count, ncclDouble, ncclSum, h->comm, h->stream));
  return 0;
}

// recv = [rank 0's count values | rank 1's | ...]
static int coll_allgather(kb_handle* h, const double* send, double* recv, size_t count) {
  if (h->lg) return local_coll(h, send, recv, count, true);
  KB_NCCL(ncclAllGather(send, recv, count, ncclDouble, h->comm, h->stream));
  return 0;
}

// error channel shared with the spline translation unit (kb_spline.hip)
namespace kb_internal {
int fail(const std::string& m) {
  g_err = m;
  return -1;
}
}  // namespace kb_internal

// replace a device buffer by a larger one, its first `keep` elements copied and the rest zero (kb_append_frames)
template <class T>
static int regrow(kb_handle* h, T** p, size_t n_new, size_t keep) {
  using U = typename std::remove_const<T>::type;
  void* q = nullptr;
  const size_t bytes = std::max<size_t>(n_new, 1) * sizeof(T);
  KB_HIP(hipMalloc(&q, bytes));
  KB_HIP(hipMemsetAsync(q, 0, bytes, h->stream));
  void* old = (void*)const_cast<U*>(*p);
  if (old && keep) KB_HIP(hipMemcpyAsync(q, old, keep * sizeof(T), hipMemcpyDeviceToDevice, h->stream));
  if (old) {
    KB_HIP(hipStreamSynchronize(h->stream));  // the copy is done before the old buffer goes
    auto it = std::find(h->allocs.begin(), h->allocs.end(), old);
    if (it != h->allocs.end()) h->allocs.erase(it);
    KB_HIP(hipFree(old));
  }
  h->allocs.push_back(q);
  *p = (T*)q;
  return 0;
}

// the frame-count-dependent launch state after kb_append_frames / kb_drop_last_frames: LDS of the build kernel,
// captured graphs (their kernel arguments hold the old layout), prepared loops and the per-call system
// (the callers check build_lds_fits for the new frame count before they change the handle)
static int relayout(kb_handle* h) {
  drop_graphs(h);
  unprepare(h);
  h->sys_valid = false;
  set_frame_counts(h);
  h->lds_build = build_lds(h);
  // one partial row per build block: fewer frames can mean more blocks (one frame per block below 256 bpc frames,
  // several above), so a dropped batch may need more rows than the handle was created with
  if (h->d.nblk > h->part_rows) {
    if (regrow(h, &h->d.part, (size_t)h->d.nblk * h->d.Wr, 0)) return -1;
    h->part_rows = h->d.nblk;
  }
  KB_HIP(hipFuncSetAttribute(h->fn_build, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_build));
  KB_HIP(hipFuncSetAttribute(h->fn_build_gn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_build));
  return 0;
}

extern "C" {

const char* kb_last_error(void) { return g_err.c_str(); }

kb_handle* kb_create(const kb_layout* L) {
  if (!L || !L->cam_model || !L->target_points) {
    fail("kb_create: null layout");
    return nullptr;
  }
  if (L->n_cams < 1 || L->n_cams > KB_MAX_CAMS) {
    fail("kb_create: n_cams out of range");
    return nullptr;
  }
  // n_frames >= 1 keeps nblk >= 1: k_colsum (and k_solve's staging) clamp their ungated row loads to nblk - 1, so
  // an empty shard would read part[-Wr]; a strong-scaling rank must own at least one frame
  if (L->n_frames < 1 || L->n_target < 1 || L->n_target > 65535) {
    fail("kb_create: bad n_frames / n_target");
    return nullptr;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    fail("kb_create: no HIP device available (the product path has no CPU fallback)");
    return nullptr;
  }
  kb_handle* h = new kb_handle();
  h->device = L->device;
  if (const char* e = std::getenv("KB_SCHED")) {  // measurement option: how the host waits in stream syncs
    const unsigned fl = !std::strcmp(e, "spin") ? hipDeviceScheduleSpin
                        : !std::strcmp(e, "yield") ? hipDeviceScheduleYield
                        : !std::strcmp(e, "block") ? hipDeviceScheduleBlockingSync : hipDeviceScheduleAuto;
    hipSetDevice(h->device);
    hipSetDeviceFlags(fl);
  }
  if (hipSetDevice(h->device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    fail("kb_create: cannot select device / create stream");
    delete h;
    return nullptr;
  }
  h->N = L->n_cams;
  h->F = L->n_frames;
  h->K = L->n_target;
  KbDev& d = h->d;
  d.N = h->N;
  d.F = h->F;
  d.K = h->K;
  int c = 0;
  for (int i = 0; i < h->N; ++i) {
    const int n = nintr_host(L->cam_model[i]);
    if (n < 0) {
      fail("kb_create: unknown camera model");
      delete h;
      return nullptr;
    }
    d.model[i] = L->cam_model[i];
    d.nintr[i] = n;
    d.col_intr[i] = c;
    c += n;
  }
  for (int j = 0; j < h->N - 1; ++j) {
    d.col_base[j] = c;
    c += 6;
  }
  h->C = c;
  if (h->C > 111) {  // [Y | z] Schur tiles: ceil((C + 1) / 16) <= 7 (7 tiles per wave of 4)
    fail("kb_create: camera block C > 111 not supported");
    delete h;
    return nullptr;
  }
  h->W = h->C * (h->C + 1) / 2 + h->C;
  d.C = h->C;
  d.off_base = h->N * KB_MAX_INTR;
  d.off_frame = h->N * KB_MAX_INTR + 7 * (h->N - 1);
  d.nsplit = std::max(1, (4 + h->N - 1) / h->N);  // >= 4 waves per build block
  d.wpb = h->N * d.nsplit;
  h->WPB = d.wpb;
  // one wave per camera and at most kBuildpMaxCams cameras: the pipelined build (N view waves + 2 frame waves);
  // KB_BUILD_PIPE=0 keeps k_build for comparison
  h->build_pipe = d.nsplit == 1 && h->N <= kBuildpMaxCams;
  if (const char* e = std::getenv("KB_BUILD_PIPE")) h->build_pipe = h->build_pipe && std::atoi(e) != 0;
  const int nbz0 = (h->C + 16) / 16, nf = (nbz0 * (nbz0 + 1) / 2 + 1) / 2 <= 5 ? 2 : 4;  // k_buildp frame waves
  h->build_threads = 64 * (h->build_pipe ? h->N + nf : d.wpb);
  if (h->build_pipe) {
    // all blocks resident at once: one block per CU (two for rigs whose block fits twice: 12 waves per CU at the
    // kernel's <= 168 VGPRs, half the LDS), each running its frames through the pipeline
    // rigs whose view role compiles several projection models and whose block has <= 8 waves use the 8-wave
    // (256-VGPR, spill-free) build kernel, one block per CU; KB_BUILDP_WIDE=0 keeps the 12-wave variant
    unsigned mm0 = 0;
    for (int i = 0; i < h->N; ++i) mm0 |= 1u << d.model[i];
    h->buildp_wide = __builtin_popcount(mm0) >= 2 && h->N + nf <= 8;
    if (const char* e = std::getenv("KB_BUILDP_WIDE")) h->buildp_wide = h->buildp_wide && std::atoi(e) != 0;
    h->bpc = (h->N + nf <= 6 && !h->buildp_wide) ? 2 : 1;
  }
  set_frame_counts(h);
  h->F_cap = h->F;
  d.W = h->W;
  d.Wp = h->N * 136 + h->W + 1;
  d.Wr = d.Wp + 1;
  d.Wtot = d.Wp + 1;  // + per-rank max|dx_f| column(s); kb_comm_init widens it to nranks
  d.nranks = 1;
  d.rank = 0;
  if (64 * d.wpb > 512) {
    fail("kb_create: camera block / rig too large for the build kernel");
    delete h;
    return nullptr;
  }

  int rc = 0;
  double* tgt = nullptr;
  rc |= h->alloc(&tgt, 3 * (size_t)h->K);
  rc |= h->alloc(&d.state, 2 * (size_t)d.S);
  rc |= h->alloc(&d.camL, 2 * 12 * (size_t)h->N);  // [2] slots: ping-pong with the state buffers
  rc |= h->alloc(&d.camK, 2 * 36 * (size_t)h->N * h->N);
  rc |= h->alloc(&d.Hff, 36 * (size_t)h->F);
  rc |= h->alloc(&d.Hfc, 6 * (size_t)h->C * h->F);
  rc |= h->alloc(&d.gf, 6 * (size_t)h->F);
  rc |= h->alloc(&d.Af, 6 * (size_t)h->C * h->F);
  rc |= h->alloc(&d.bf, 6 * (size_t)h->F);
  rc |= h->alloc(&d.part, (size_t)d.nblk * d.Wr);
  h->part_rows = d.nblk;
  rc |= h->alloc(&d.part8, (size_t)kColsumRows * d.Wtot);
  rc |= h->alloc(&d.psum_local, (size_t)d.Wtot);
  d.psum = d.psum_local;
  d.psum_rows = 1;
  // the pass end runs in its own one-block kernel (k_post), not folded into the next k_build: a folded end has block 0
  // store the new control block while the other blocks load it, and under k_build's L2 pressure a block on another
  // XCD can read it torn across cache lines (seen once as a diverged LM run on configs[3])
  d.fold = 0;
  if (const char* e = std::getenv("KB_GN_FUSED")) h->gn_fuse = std::atoi(e) != 0;
  d.dbg_stop = -1;
  d.dbg_flags = 0;
  rc |= h->alloc(&d.ticket, 16);
  rc |= h->alloc(&d.Hcc, (size_t)h->C * h->C);
  rc |= h->alloc(&d.gc, (size_t)h->C);
  rc |= h->alloc(&d.cost_build, 2);
  rc |= h->alloc(&d.dx, (size_t)h->ncols);
  rc |= h->alloc(&d.rhs, (size_t)h->ncols);
  rc |= h->alloc(&d.bpart, 4 * (size_t)d.nblk_bs);
  d.bsrc = d.bpart;
  d.bsrc_rows = d.nblk_bs;
  rc |= h->alloc(&d.camstat, 4);
  rc |= h->alloc(&d.red_local, 8);
  d.red = d.red_local;
  rc |= h->alloc(&d.ctrl, 1);
  if (h->C > 64) {  // k_solve's staged camera block (k_colimg / k_colsumx), sized as in the LDS budget below
    const int nb = (h->C + 16) / 16;  // rows 0 .. C: the right-hand side is appended as row C
    rc |= h->alloc(&d.simg, (size_t)kTileSz * nb * (nb + 1) / 2 + 16 * nb + 2 + kXMaxRanks);
  }
  std::vector<int32_t> colinfo(h->C), tri(h->C * (h->C + 1) / 2);
  for (int i = 0; i < h->N; ++i)
    for (int x = 0; x < d.nintr[i]; ++x) colinfo[d.col_intr[i] + x] = (0 << 16) | (i << 8) | x;
  for (int j = 0; j < h->N - 1; ++j)
    for (int x = 0; x < 6; ++x) colinfo[d.col_base[j] + x] = (1 << 16) | (j << 8) | x;
  int e = 0;
  for (int a = 0; a < h->C; ++a)
    for (int b = a; b < h->C; ++b) tri[e++] = (a << 16) | b;
  int32_t *ci = nullptr, *tr = nullptr;
  rc |= h->alloc(&ci, colinfo.size());
  rc |= h->alloc(&tr, tri.size());
  if (rc) {
    kb_destroy(h);
    return nullptr;
  }
  d.colinfo = ci;
  d.tri = tr;
  d.target = tgt;
  hipMemcpyAsync(ci, colinfo.data(), colinfo.size() * sizeof(int32_t), hipMemcpyHostToDevice, h->stream);
  hipMemcpyAsync(tr, tri.data(), tri.size() * sizeof(int32_t), hipMemcpyHostToDevice, h->stream);
  hipMemcpyAsync(tgt, L->target_points, 3 * sizeof(double) * h->K, hipMemcpyHostToDevice, h->stream);
  {
    const int N = h->N, C = h->C, WPB = d.wpb;
    const int CZ = 16 * ((C + 16) / 16);  // [Y | z] row stride of the Schur tiles
    (void)WPB;
    h->lds_build = build_lds(h);
    h->lds_camexp = sizeof(double) * (N * 256 + N * N * 36);
    h->lds_schur = sizeof(double) * 16 * CZ;
    if (C <= 64) {
      h->lds_solve = sizeof(double) * (C * (C + 1) / 2 + 2 * C + 1 + N * 256 + 2 * N * N * 36) + sizeof(int) * C;
    } else {  // the k_colimg image (complete system: 16 x 16 lower tiles, b as row C | g_c) + the factored diagonal
      // tiles and their inverses + 1/D
      const int nb = (C + 16) / 16, n16 = 16 * nb;
      // tiles | aux: g_c (n16, non-PD count at C) | cost | max|dx_f| per rank (expanded partials) | pad
      d.img_n = kTileSz * nb * (nb + 1) / 2 + n16 + 2 + kXMaxRanks;
      h->lds_solve = sizeof(double) * (d.img_n + 2 + 2 * nb * kTileSz + n16) + sizeof(int) * C;
      h->lds_colimg = sizeof(double) * (N * 256 + 2 * N * N * 36) + sizeof(int) * C;
    }
    h->solve_threads = C <= 64 ? 256 : 512;
    // expanded partials for the GN fused loop: k_buildp expands its own camera sums in the LDS its view tiles free
    // (Hs [N][256] | T [N(N-1)/2][36] | H_cc, g_c [W] within the Xw + Hw regions); KB_XEXP=0 keeps k_colimg
    h->xexp = C > 64 && h->build_pipe && N * 256 + 18 * N * (N - 1) + h->W <= N * 64 * XS + N * 256;
    if (const char* e = std::getenv("KB_XEXP")) h->xexp = h->xexp && std::atoi(e) != 0;
    h->fn_solve = C <= 16   ? (const void*)k_solve<16>
                  : C <= 24 ? (const void*)k_solve<24>
                  : C <= 32 ? (const void*)k_solve<32>
                  : C <= 48 ? (const void*)k_solve<48>
                  : C <= 64 ? (const void*)k_solve<64>
                            : (const void*)k_solve<0>;
    if (h->lds_build + (h->build_pipe ? kBuildpStaticLds : 0) > 160 * 1024 || h->lds_solve > 160 * 1024 ||
        h->lds_camexp > 160 * 1024) {
      fail("kb_create: LDS budget exceeded for this rig");
      kb_destroy(h);
      return nullptr;
    }
  }
  {
    // Schur-sum tiles per wave (template bucket): ceil(lower tiles of [Y|z]^T [Y|z] / waves)
    const int nbz = (h->C + 16) / 16, ntiles = nbz * (nbz + 1) / 2;
    const int tb = (ntiles + d.wpb - 1) / d.wpb, ts = (ntiles + 3) / 4;
    h->mb = h->build_pipe ? ((ntiles + 1) / 2 <= 5 ? 5 : 7) : tb <= 1 ? 1 : tb <= 4 ? 4 : 7;
    h->ms = ts <= 1 ? 1 : ts <= 4 ? 4 : 7;
    // camera-model set: one-model rigs (and the omni-radtan + EUCM rig of configs[2]) get their own build
    // kernels; any other mix uses the all-models instantiation
    unsigned mm = 0;
    for (int i = 0; i < h->N; ++i) mm |= 1u << d.model[i];
    h->fn_build = pick_build<false>(h->mb, mm, h->build_pipe, h->buildp_wide);
    h->fn_build_gn = pick_build<true>(h->mb, mm, h->build_pipe, h->buildp_wide);
    h->fn_schur = h->ms == 1 ? (const void*)k_schur<1> : h->ms == 4 ? (const void*)k_schur<4> : (const void*)k_schur<7>;
  }
  hipFuncSetAttribute(h->fn_build, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_build);
  hipFuncSetAttribute(h->fn_build_gn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_build);
  hipFuncSetAttribute((const void*)k_camexpand, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_camexp);
  hipFuncSetAttribute(h->fn_schur, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_schur);
  hipFuncSetAttribute(h->fn_solve, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_solve);
  hipFuncSetAttribute((const void*)k_colimg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_colimg);
  if (hipStreamSynchronize(h->stream) != hipSuccess) {
    fail("kb_create: stream sync failed");
    kb_destroy(h);
    return nullptr;
  }
  return h;
}

void kb_destroy(kb_handle* h) {
  if (!h) return;
  hipSetDevice(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  drop_graphs(h);
  for (void* p : h->xar_opened) hipIpcCloseMemHandle(p);
  if (h->comm) ncclCommDestroy(h->comm);
  if (h->lg && --h->lg->refs == 0) {
    for (auto e : h->lg->ready) hipEventDestroy(e);
    for (auto e : h->lg->done) hipEventDestroy(e);
    delete h->lg;
  }
  for (void* p : h->allocs) hipFree(p);
  if (h->trace) hipFree(h->trace);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
}

int kb_state_size(const kb_handle* h) { return h ? h->S : -1; }
int kb_num_cols(const kb_handle* h) { return h ? h->ncols : -1; }
int kb_camera_cols(const kb_handle* h) { return h ? h->C : -1; }

int kb_upload_observations(kb_handle* h, int32_t n_views, int32_t n_corners, const double* y, const uint16_t* corner_id,
                           const uint32_t* view_offsets, const uint32_t* view_frame, const uint8_t* view_cam) {
  if (!h) return fail("null handle");
  if (h->uploaded) return fail("kb_upload_observations: observations already uploaded for this handle");
  if (n_views < 1 || n_corners < 1 || !y || !corner_id || !view_offsets || !view_frame || !view_cam)
    return fail("kb_upload_observations: empty or null input");
  KB_HIP(hipSetDevice(h->device));
  // host-side validation: shapes the kernels and grids assume
  if (view_offsets[0] != 0 || (int64_t)view_offsets[n_views] != n_corners)
    return fail("kb_upload_observations: view_offsets must start at 0 and end at n_corners");
  std::vector<int32_t> fvc((size_t)h->F * h->N, -1), vf(n_views), vc(n_views);
  for (int v = 0; v < n_views; ++v) {
    if (view_offsets[v + 1] < view_offsets[v]) return fail("kb_upload_observations: view_offsets not monotone");
    if ((int)view_frame[v] >= h->F || view_cam[v] >= h->N) return fail("kb_upload_observations: view index out of range");
    if (v > 0 && view_frame[v] < view_frame[v - 1]) return fail("kb_upload_observations: views must be sorted by frame");
    int32_t& slot = fvc[(size_t)view_frame[v] * h->N + view_cam[v]];
    if (slot >= 0) return fail("kb_upload_observations: two views for one (frame, camera)");
    slot = v;
    vf[v] = (int32_t)view_frame[v];
    vc[v] = (int32_t)view_cam[v];
  }
  for (int k = 0; k < n_corners; ++k)
    if ((int)corner_id[k] >= h->K) return fail("kb_upload_observations: corner_id out of range");
  h->V = n_views;
  h->NC = n_corners;
  h->vcam.assign(vc.begin(), vc.end());
  h->V_cap = n_views;
  h->NC_cap = n_corners;
  h->vo_host.assign(view_offsets, view_offsets + n_views + 1);
  h->frame_v0.assign(h->F + 1, n_views);
  for (int v = n_views - 1; v >= 0; --v) h->frame_v0[vf[v]] = v;
  for (int f = h->F - 1; f >= 0; --f) h->frame_v0[f] = std::min(h->frame_v0[f], h->frame_v0[f + 1]);
  KbDev& d = h->d;
  d.V = n_views;
  d.NC = n_corners;
  d.nblk_cost = (n_views + 3) / 4;
  double2* yd = nullptr;
  uint16_t* cd = nullptr;
  uint32_t* vo = nullptr;
  int32_t *vfd = nullptr, *vcd = nullptr, *fv = nullptr;
  int rc = 0;
  rc |= h->alloc(&yd, (size_t)n_corners);
  rc |= h->alloc(&cd, (size_t)n_corners);
  rc |= h->alloc(&vo, (size_t)n_views + 1);
  rc |= h->alloc(&vfd, (size_t)n_views);
  rc |= h->alloc(&vcd, (size_t)n_views);
  rc |= h->alloc(&fv, fvc.size());
  int2* fvo = nullptr;
  rc |= h->alloc(&fvo, fvc.size());
  rc |= h->alloc(&d.costpart, (size_t)d.nblk_cost);
  if (rc) return -1;
  KB_HIP(hipMemcpyAsync(yd, y, sizeof(double2) * n_corners, hipMemcpyHostToDevice, h->stream));
  KB_HIP(hipMemcpyAsync(cd, corner_id, sizeof(uint16_t) * n_corners, hipMemcpyHostToDevice, h->stream));
  KB_HIP(hipMemcpyAsync(vo, view_offsets, sizeof(uint32_t) * (n_views + 1), hipMemcpyHostToDevice, h->stream));
  KB_HIP(hipMemcpyAsync(vfd, vf.data(), sizeof(int32_t) * n_views, hipMemcpyHostToDevice, h->stream));
  KB_HIP(hipMemcpyAsync(vcd, vc.data(), sizeof(int32_t) * n_views, hipMemcpyHostToDevice, h->stream));
  KB_HIP(hipMemcpyAsync(fv, fvc.data(), sizeof(int32_t) * fvc.size(), hipMemcpyHostToDevice, h->stream));
  std::vector<int2> fvr(fvc.size());
  for (size_t q = 0; q < fvc.size(); ++q)
    fvr[q] = fvc[q] < 0 ? make_int2(0, 0)
                        : make_int2((int)view_offsets[fvc[q]], (int)view_offsets[fvc[q] + 1]);
  KB_HIP(hipMemcpyAsync(fvo, fvr.data(), sizeof(int2) * fvr.size(), hipMemcpyHostToDevice, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  d.y = yd;
  d.cid = cd;
  d.view_off = vo;
  d.view_frame = vfd;
  d.view_cam = vcd;
  d.frame_vcam = fv;
  d.fview = fvo;
  h->uploaded = true;
  return 0;
}

int kb_append_frames(kb_handle* h, int32_t n_frames, int32_t n_views, int32_t n_corners, const double* y,
                     const uint16_t* corner_id, const uint32_t* view_offsets, const uint32_t* view_frame,
                     const uint8_t* view_cam, const double* frame_poses) {
  if (!h) return fail("kb_append_frames: null handle");
  if (!h->uploaded) return fail("kb_append_frames: no observations (kb_upload_observations first)");
  if (sharded(h)) return fail("kb_append_frames: not available on a sharded handle");
  const int nf = n_frames, nv = n_views, nc = n_corners;
  if (nf < 1 || nv < 0 || nc < 0 || !frame_poses || (nv > 0 && (!view_offsets || !view_frame || !view_cam)) ||
      (nc > 0 && (!y || !corner_id)))
    return fail("kb_append_frames: bad arguments");
  if (nv == 0 ? nc != 0 : (view_offsets[0] != 0 || (int64_t)view_offsets[nv] != nc))
    return fail("kb_append_frames: view_offsets must start at 0 and end at n_corners");
  KB_HIP(hipSetDevice(h->device));
  const int N = h->N, F0 = h->F, V0 = h->V, NC0 = h->NC;
  // host-side validation of the appended block (frames 0 .. nf - 1 of it), as kb_upload_observations
  std::vector<int32_t> fvc((size_t)nf * N, -1), vfg(nv), vcg(nv);
  std::vector<int2> fvr((size_t)nf * N, make_int2(0, 0));
  std::vector<uint32_t> vog(nv);
  for (int v = 0; v < nv; ++v) {
    if (view_offsets[v + 1] < view_offsets[v]) return fail("kb_append_frames: view_offsets not monotone");
    if ((int)view_frame[v] >= nf || view_cam[v] >= N) return fail("kb_append_frames: view index out of range");
    if (v > 0 && view_frame[v] < view_frame[v - 1]) return fail("kb_append_frames: views must be sorted by frame");
    int32_t& slot = fvc[(size_t)view_frame[v] * N + view_cam[v]];
    if (slot >= 0) return fail("kb_append_frames: two views for one (frame, camera)");
    slot = V0 + v;
    fvr[(size_t)view_frame[v] * N + view_cam[v]] = make_int2(NC0 + (int)view_offsets[v], NC0 + (int)view_offsets[v + 1]);
    vfg[v] = F0 + (int32_t)view_frame[v];
    vcg[v] = view_cam[v];
    vog[v] = (uint32_t)NC0 + view_offsets[v + 1];
  }
  for (int k = 0; k < nc; ++k)
    if ((int)corner_id[k] >= h->K) return fail("kb_append_frames: corner_id out of range");
  KbDev& d = h->d;
  const int F1 = F0 + nf, V1 = V0 + nv, NC1 = NC0 + nc;
  // a rejected append leaves the handle as it was: the layout is checked before anything changes, and a failed
  // regrow below only leaves some buffers larger (their contents kept where they matter), never a new frame count
  if (!build_lds_fits(h, F1)) return fail("kb_append_frames: build-kernel LDS budget exceeded for this frame count");
  // buffers may move from here on: the captured graphs' arguments would hold freed ones (recaptured on next use)
  drop_graphs(h);
  h->sys_valid = false;
  // capacities: geometric growth, so a sequence of single-frame appends moves O(F) data in total
  if (F1 > h->F_cap) {
    const size_t fc = std::max(F1, 2 * h->F_cap), C = h->C;
    const bool bad = regrow(h, &d.Hff, 36 * fc, 0) || regrow(h, &d.Hfc, 6 * C * fc, 0) || regrow(h, &d.gf, 6 * fc, 0) ||
                     regrow(h, &d.Af, 6 * C * fc, 0) || regrow(h, &d.bf, 6 * fc, 0) ||
                     regrow(h, &d.dx, C + 6 * fc, 0) || regrow(h, &d.rhs, C + 6 * fc, 0) ||
                     regrow(h, &d.bpart, 4 * fc, 0) || regrow(h, &d.fview, fc * N, (size_t)F0 * N) ||
                     regrow(h, &d.frame_vcam, fc * N, (size_t)F0 * N);
    d.bsrc = d.bpart;  // whether or not every buffer grew: bsrc never points at a freed one
    if (bad) return -1;
    if ((size_t)h->part_rows < fc) {
      if (regrow(h, &d.part, fc * d.Wr, 0)) return -1;
      h->part_rows = (int)fc;
    }
    d.bsrc_rows = (int)fc;  // rows beyond F are never read (k_post reduces nblk_bs = F rows)
    h->F_cap = (int)fc;
  }
  const int base = N * KB_MAX_INTR + 7 * (N - 1), S0 = h->S;
  if (base + 7 * F1 > d.S) {  // the state's slot stride grows: both slots move into a larger buffer
    const int sst = base + 7 * h->F_cap;
    void* q = nullptr;
    KB_HIP(hipMalloc(&q, 2 * (size_t)sst * sizeof(double)));
    KB_HIP(hipMemsetAsync(q, 0, 2 * (size_t)sst * sizeof(double), h->stream));
    for (int sl = 0; sl < 2; ++sl)
      KB_HIP(hipMemcpyAsync((double*)q + (size_t)sl * sst, d.state + (size_t)sl * d.S, sizeof(double) * S0,
                            hipMemcpyDeviceToDevice, h->stream));
    KB_HIP(hipStreamSynchronize(h->stream));
    auto it = std::find(h->allocs.begin(), h->allocs.end(), (void*)d.state);
    if (it != h->allocs.end()) h->allocs.erase(it);
    KB_HIP(hipFree(d.state));
    h->allocs.push_back(q);
    d.state = (double*)q;
    d.S = sst;
  }
  if (V1 > h->V_cap) {
    const size_t vc = std::max(V1, 2 * h->V_cap);
    if (regrow(h, &d.view_off, vc + 1, (size_t)V0 + 1) || regrow(h, &d.view_frame, vc, (size_t)V0) ||
        regrow(h, &d.view_cam, vc, (size_t)V0) || regrow(h, &d.costpart, (vc + 3) / 4, 0))
      return -1;
    h->V_cap = (int)vc;
  }
  if (NC1 > h->NC_cap) {
    const size_t ncc = std::max(NC1, 2 * h->NC_cap);
    if (regrow(h, &d.y, ncc, (size_t)NC0) || regrow(h, &d.cid, ncc, (size_t)NC0)) return -1;
    h->NC_cap = (int)ncc;
  }
  // only the new observations cross PCIe
  if (nc > 0) {
    KB_HIP(hipMemcpyAsync(const_cast<double2*>(d.y) + NC0, y, sizeof(double2) * nc, hipMemcpyHostToDevice, h->stream));
    KB_HIP(hipMemcpyAsync(const_cast<uint16_t*>(d.cid) + NC0, corner_id, sizeof(uint16_t) * nc, hipMemcpyHostToDevice,
                          h->stream));
  }
  if (nv > 0) {
    KB_HIP(hipMemcpyAsync(const_cast<uint32_t*>(d.view_off) + V0 + 1, vog.data(), sizeof(uint32_t) * nv,
                          hipMemcpyHostToDevice, h->stream));
    KB_HIP(hipMemcpyAsync(const_cast<int32_t*>(d.view_frame) + V0, vfg.data(), sizeof(int32_t) * nv,
                          hipMemcpyHostToDevice, h->stream));
    KB_HIP(hipMemcpyAsync(const_cast<int32_t*>(d.view_cam) + V0, vcg.data(), sizeof(int32_t) * nv,
                          hipMemcpyHostToDevice, h->stream));
  }
  KB_HIP(hipMemcpyAsync(const_cast<int32_t*>(d.frame_vcam) + (size_t)F0 * N, fvc.data(), sizeof(int32_t) * fvc.size(),
                        hipMemcpyHostToDevice, h->stream));
  KB_HIP(hipMemcpyAsync(const_cast<int2*>(d.fview) + (size_t)F0 * N, fvr.data(), sizeof(int2) * fvr.size(),
                        hipMemcpyHostToDevice, h->stream));
  // the new frames' poses (initial guesses) into the current state buffer
  KB_HIP(hipMemcpyAsync(d.state + (size_t)h->cur * d.S + base + 7 * F0, frame_poses, sizeof(double) * 7 * nf,
                        hipMemcpyHostToDevice, h->stream));
  h->F = F1;
  h->V = V1;
  h->NC = NC1;
  d.V = V1;
  d.NC = NC1;
  d.nblk_cost = (V1 + 3) / 4;
  for (int v = 0; v < nv; ++v) h->vcam.push_back(vcg[v]);
  h->vo_host.insert(h->vo_host.end(), vog.begin(), vog.end());
  h->frame_v0.resize(F1 + 1, V1);
  for (int f = F1 - 1; f >= F0; --f) h->frame_v0[f] = h->frame_v0[f + 1];
  for (int v = nv - 1; v >= 0; --v) h->frame_v0[vfg[v]] = V0 + v;
  for (int f = F1 - 1; f >= F0; --f) h->frame_v0[f] = std::min(h->frame_v0[f], h->frame_v0[f + 1]);
  if (relayout(h)) return -1;
  KB_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kb_drop_last_frames(kb_handle* h, int32_t n_frames) {
  if (!h) return fail("kb_drop_last_frames: null handle");
  if (!h->uploaded) return fail("kb_drop_last_frames: no observations");
  if (sharded(h)) return fail("kb_drop_last_frames: not available on a sharded handle");
  if (n_frames < 1 || n_frames >= h->F) return fail("kb_drop_last_frames: must keep at least one frame");
  KB_HIP(hipSetDevice(h->device));
  const int F1 = h->F - n_frames, V1 = h->frame_v0[F1], NC1 = (int)h->vo_host[V1];
  if (!build_lds_fits(h, F1)) return fail("kb_drop_last_frames: build-kernel LDS budget exceeded for this frame count");
  {  // fewer frames can mean more build blocks: the partial rows grow first, so a failure leaves the handle as it was
    const int g1 = gframes_for(h, F1), nblk1 = (F1 + g1 - 1) / g1;
    if (nblk1 > h->part_rows) {
      if (regrow(h, &h->d.part, (size_t)nblk1 * h->d.Wr, 0)) return -1;
      h->part_rows = nblk1;
    }
  }
  h->F = F1;
  h->V = V1;
  h->NC = NC1;
  h->d.V = V1;
  h->d.NC = NC1;
  h->d.nblk_cost = (V1 + 3) / 4;
  h->vcam.resize(V1);
  h->vo_host.resize(V1 + 1);
  h->frame_v0.resize(F1 + 1);
  h->frame_v0[F1] = V1;
  return relayout(h);
}

static int set_cur(kb_handle* h, int cur) {
  h->cur = cur;
  KB_HIP(hipMemcpyAsync(&h->d.ctrl->cur, &h->cur, sizeof(int), hipMemcpyHostToDevice, h->stream));
  return 0;
}

int kb_set_state_flat(kb_handle* h, const double* state) {
  if (!h || !state) return fail("kb_set_state_flat: null");
  KB_HIP(hipSetDevice(h->device));
  unprepare(h);
  KB_HIP(hipMemcpyAsync(h->d.state + (size_t)h->cur * h->d.S, state, sizeof(double) * h->S, hipMemcpyHostToDevice,
                        h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kb_set_state(kb_handle* h, const double* poses_q, const double* poses_t, const double* baselines,
                 const double* intrinsics) {
  if (!h || !poses_q || !poses_t || !intrinsics || (h->N > 1 && !baselines)) return fail("kb_set_state: null");
  std::vector<double> s(h->S, 0.0);
  for (int q = 0; q < h->N * KB_MAX_INTR; ++q) s[q] = intrinsics[q];
  for (int q = 0; q < 7 * (h->N - 1); ++q) s[h->d.off_base + q] = baselines[q];
  for (int f = 0; f < h->F; ++f) {
    for (int q = 0; q < 4; ++q) s[h->d.off_frame + 7 * f + q] = poses_q[4 * f + q];
    for (int q = 0; q < 3; ++q) s[h->d.off_frame + 7 * f + 4 + q] = poses_t[3 * f + q];
  }
  return kb_set_state_flat(h, s.data());
}

int kb_get_state_flat(kb_handle* h, double* state) {
  if (!h || !state) return fail("kb_get_state_flat: null");
  KB_HIP(hipSetDevice(h->device));
  KB_HIP(hipMemcpyAsync(state, h->d.state + (size_t)h->cur * h->d.S, sizeof(double) * h->S, hipMemcpyDeviceToHost,
                        h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

// ---------------------------------------------------------------- launch helpers
static int launch_cost(kb_handle* h, int which) {
  hipLaunchKernelGGL(k_cost, dim3(h->d.nblk_cost), dim3(256), 0, h->stream, h->d, which);
  hipLaunchKernelGGL(k_reduce_cost, dim3(1), dim3(256), 0, h->stream, h->d);
  KB_HIP(hipGetLastError());
  return 0;
}

// one all-gather of every rank's [cost, dx.dx, dx.rhs, max|dx|]; reduced in rank order on every rank (by
// k_red_gather, or inline by k_policy) so that all ranks hold bitwise-identical sums
static int allreduce_red(kb_handle* h, bool reduce = true) {
  if (!sharded(h)) return 0;
  if (coll_allgather(h, h->d.red_local, const_cast<double*>(h->d.red_all), 4)) return -1;
  if (reduce) {
    hipLaunchKernelGGL(k_red_gather, dim3(1), dim3(1), 0, h->stream, h->d);
    KB_HIP(hipGetLastError());
  }
  return 0;
}

// column sums of the block partials (finished in-kernel) + all-reduce over ranks when sharded
// finish = 0 (one GPU, optimizer loop): k_solve sums the kColsumRows stage-1 rows itself
// finish = 0 (optimizer loop): the consumer (k_solve) sums the kColsumRows stage-1 rows; sharded, those rows are
// all-reduced as they are (one collective, no finishing kernel)
static int launch_colsum(kb_handle* h, int gate, bool finish = true) {
  KbDev& d = h->d;
  if (d.xexp) {
    // expanded partials (GN fused, C > 64): the column sums go straight into the k_solve image (this rank's partial
    // image when sharded, all-reduced into simg: 62 KB at configs[3])
    const int nx = (h->C + 1) + (d.Wtot - h->N * 136);
    hipLaunchKernelGGL(k_colsumx, dim3((nx + 63) / 64), dim3(64 * kColsum1Waves), 0, h->stream, d, gate);
    KB_HIP(hipGetLastError());
    if (sharded(h)) {
      if (d.xar) {  // direct: every rank sums the ranks' partial images itself (k_xar)
        hipLaunchKernelGGL(k_xar, dim3(kXarBlocks), dim3(256), 0, h->stream, d, gate);
        KB_HIP(hipGetLastError());
      } else if (coll_allreduce(h, h->ximg_part, d.simg, d.img_n)) {
        return -1;
      }
    }
    return 0;
  }
  if (finish && h->C > 64) {
    // camera blocks for the tiled solve: the block partials summed in one pass into one row (k_colsum1), then
    // k_colimg copies the sums (into the consumer's row) and writes k_solve's LDS image from that row.  Sharded,
    // the ranks all-reduce the single row (55 KB at configs[3])
    hipLaunchKernelGGL(k_colsum1, dim3((d.Wtot + 63) / 64), dim3(64 * kColsum1Waves), 0, h->stream, d, gate);
    KB_HIP(hipGetLastError());
    const double* rows = d.part8;
    const int nrows = 1;
    if (sharded(h)) {
      if (coll_allreduce(h, d.part8, h->psum_red8, d.Wtot)) return -1;
      rows = h->psum_red8;
    }
    double* out = sharded(h) ? h->psum_red : d.psum_local;
    hipLaunchKernelGGL(k_colimg, dim3((d.Wtot + d.img_n + kColimgThreads - 1) / kColimgThreads), dim3(kColimgThreads),
                       h->lds_colimg, h->stream, d, rows, out, gate, nrows);
    KB_HIP(hipGetLastError());
    return 0;
  }
  hipLaunchKernelGGL(k_colsum, dim3((d.Wtot + 63) / 64, kColsumRows), dim3(256), 0, h->stream, d, gate);
  if (finish) hipLaunchKernelGGL(k_colfin, dim3((d.Wtot + 255) / 256), dim3(256), 0, h->stream, d, gate);
  KB_HIP(hipGetLastError());
  if (sharded(h)) {
    if (finish ? coll_allreduce(h, d.psum_local, h->psum_red, d.Wtot)
               : coll_allreduce(h, d.part8, h->psum_red8, (size_t)kColsumRows * d.Wtot))
      return -1;
  }
  return 0;
}

static int launch_build(kb_handle* h, int gate, int fuse) {
  KbDev& d = h->d;
  // per-call path: camera chains first; in the loop k_solve (or the loop start) computed them
  if (!gate) hipLaunchKernelGGL(k_pre, dim3(1), dim3(256), 0, h->stream, d, 0);
  void* args[] = {&d, &gate, &fuse};
  KB_HIP(hipLaunchKernel(d.gn_fused ? h->fn_build_gn : h->fn_build, dim3(d.nblk), dim3(h->build_threads), args,
                         h->lds_build, h->stream));
  return 0;
}

static int launch_schur(kb_handle* h, int gate) {
  void* args[] = {&h->d, &gate};
  KB_HIP(hipLaunchKernel(h->fn_schur, dim3(h->d.nblk), dim3(256), args, h->lds_schur, h->stream));
  KB_HIP(hipGetLastError());
  return 0;
}

static int launch_solve(kb_handle* h, int gate, int do_update, bool from_rows = false) {
  KbDev d = h->d;
  if (from_rows) {  // column sums still split in kColsumRows stage-1 rows (all-reduced ones when sharded)
    d.psum = sharded(h) ? h->psum_red8 : d.part8;
    d.psum_rows = kColsumRows;
  }
  void* args[] = {(void*)&d, (void*)&gate, (void*)&do_update};
  KB_HIP(hipLaunchKernel(h->fn_solve, dim3(1), dim3(h->solve_threads), args, h->lds_solve, h->stream));
  KB_HIP(hipGetLastError());
  return 0;
}

static int launch_backsub(kb_handle* h, int gate, int do_update, int with_cost) {
  hipLaunchKernelGGL(k_backsub, dim3((h->F + kBsFrames - 1) / kBsFrames), dim3(64 * kBsFrames), 0, h->stream, h->d, gate,
                     do_update, with_cost);
  KB_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------- per-call API
int kb_eval_cost(kb_handle* h, double* J_out) {
  if (!h || !J_out) return fail("kb_eval_cost: null");
  if (!h->uploaded) return fail("kb_eval_cost: no observations");
  KB_HIP(hipSetDevice(h->device));
  unprepare(h);  // writes red / the cost partials the prepared loop start left
  if (launch_cost(h, 0)) return -1;
  if (allreduce_red(h)) return -1;
  KB_HIP(hipMemcpyAsync(J_out, h->d.red, sizeof(double), hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kb_build(kb_handle* h, int use_mestimator) {
  if (!h) return fail("kb_build: null");
  if (!h->uploaded) return fail("kb_build: no observations");
  (void)use_mestimator;  // NoMEstimator: weight 1 either way (ErrorTerm.cpp:11)
  KB_HIP(hipSetDevice(h->device));
  unprepare(h);
  h->sys_valid = false;
  if (launch_build(h, 0, 0)) return -1;
  if (launch_colsum(h, 0)) return -1;
  hipLaunchKernelGGL(k_camexpand, dim3(1), dim3(256), h->lds_camexp, h->stream, h->d, 0);
  KB_HIP(hipGetLastError());
  KB_HIP(hipStreamSynchronize(h->stream));
  h->sys_valid = true;
  return 0;
}

int kb_set_constant_conditioner(kb_handle* h, double diag) {
  if (!h) return fail("null handle");
  h->d.host_lambda = diag;
  h->use_cond = false;
  return 0;
}

int kb_set_conditioner(kb_handle* h, const double* diag) {
  if (!h || !diag) return fail("kb_set_conditioner: null");
  KB_HIP(hipSetDevice(h->device));
  if (h->cond_n < (size_t)h->ncols) {
    if (regrow(h, &h->cond2, (size_t)h->ncols, 0)) return -1;
    h->cond_n = (size_t)h->ncols;
  }
  std::vector<double> sq(h->ncols);
  for (int k = 0; k < h->ncols; ++k) sq[k] = diag[k] * diag[k];  // "the square of these values" (:33-35)
  KB_HIP(hipMemcpyAsync(h->cond2, sq.data(), sizeof(double) * h->ncols, hipMemcpyHostToDevice, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  h->use_cond = true;
  return 0;
}

// ---------------------------------------------------------------- block-Jacobi PCG (LinearSolverPCG)
// projection / distortion DV sizes of a camera model (CameraDesignVariable: projection, distortion DVs)
static void dv_split(int model, int* a, int* b) {
  switch (model) {
    case KB_OMNI_RADTAN: *a = 5, *b = 4; break;
    case KB_EUCM: *a = 6, *b = 0; break;
    case KB_OMNI: *a = 5, *b = 0; break;
    case KB_DS: *a = 6, *b = 0; break;
    case KB_PINHOLE_FOV: *a = 4, *b = 1; break;
    default: *a = 4, *b = 4; break;  // pinhole-radtan, pinhole-equidistant
  }
}

static size_t pcg_lds(int fpb, int C, int F) {
  const size_t R = 6 * (size_t)fpb, nblk = (F + fpb - 1) / fpb, nrow = (C + nblk - 1) / nblk;
  return sizeof(double) * (R * C + 54 * (size_t)fpb + 5 * R + 11 * (size_t)C + nrow * C) + sizeof(int) * 2 * (size_t)C;
}

// the PCG buffers and the camera DV block table (first use)
static int ensure_pcg(kb_handle* h) {
  const int C = h->C, F = h->F;
  if (h->pcg_F < (size_t)F) {  // (re)sized for the current frame count (kb_append_frames grows it)
    if (regrow(h, &h->pcg_buf, (size_t)F * (C + 1) + F + 12, 0)) return -1;
    h->pcg_F = (size_t)F;
  }
  if (!h->pcg_cb) {
    if (h->alloc(&h->pcg_cb, 2 * (size_t)C) || h->alloc(&h->pcg_bar, kPcgBarWords)) return -1;
    std::vector<int> cb(2 * C);
    int c = 0;
    auto block = [&](int m) {
      for (int k = 0; k < m; ++k) {
        cb[c + k] = c;
        cb[C + c + k] = m;
      }
      c += m;
    };
    for (int i = 0; i < h->N; ++i) {
      int a, b;
      dv_split(h->d.model[i], &a, &b);
      block(a);
      if (b) block(b);
    }
    for (int j = 0; j < h->N - 1; ++j) {
      block(3);
      block(3);
    }
    if (c != C) return fail("kb_solve (PCG): camera DV blocks do not cover the camera columns");
    KB_HIP(hipMemcpyAsync(h->pcg_cb, cb.data(), sizeof(int) * 2 * C, hipMemcpyHostToDevice, h->stream));
  }
  return 0;
}

static int run_pcg(kb_handle* h, int* ok) {
  if (sharded(h)) return fail("kb_solve (PCG): not available on a sharded handle");
  const int C = h->C, F = h->F;
  if (ensure_pcg(h)) return -1;
  // frames per block: >= 64 blocks when there are enough frames, H_fc rows of the block within ~120 KB of LDS
  int fpb = std::max(1, std::min(kPcgMaxFpb, (F + 63) / 64));
  while (fpb > 1 && pcg_lds(fpb, C, F) > 120 * 1024) --fpb;
  const size_t lds = pcg_lds(fpb, C, F);
  const int nblk = (F + fpb - 1) / fpb;
  int per_cu = 0, ncu = 0;
  KB_HIP(hipFuncSetAttribute((const void*)k_pcg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  KB_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_pcg, kPcgThreads, lds));
  KB_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, h->device));
  if (lds > 160 * 1024 || per_cu < 1 || nblk > per_cu * ncu)
    return fail("kb_solve (PCG): problem too large for one co-resident grid");
  KbPcg P;
  P.lam2 = h->d.host_lambda * h->d.host_lambda;
  P.tol = h->pcg.tolerance;
  P.prev_residual = h->pcg_residual;
  P.max_it = h->pcg.max_iterations < 0 ? h->ncols : h->pcg.max_iterations;
  P.abs_tol = h->pcg.absolute_tolerance ? 1 : 0;
  P.fpb = fpb;
  P.nblk = nblk;
  P.cb_start = h->pcg_cb;
  P.cb_size = h->pcg_cb + C;
  P.part = h->pcg_buf;
  P.part2 = P.part + (size_t)F * (C + 1);
  P.info = P.part2 + F;
  P.bar = h->pcg_bar;
  KB_HIP(hipMemsetAsync(h->pcg_bar, 0, sizeof(unsigned) * kPcgBarWords, h->stream));
  KB_HIP(hipMemsetAsync(P.info, 0, sizeof(double) * 8, h->stream));
  void* args[] = {(void*)&h->d, (void*)&P};
  KB_HIP(hipLaunchCooperativeKernel((const void*)k_pcg, dim3(nblk), dim3(kPcgThreads), args, (unsigned)lds,
                                    h->stream));
  double info[8];
  KB_HIP(hipMemcpyAsync(info, P.info, sizeof(info), hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  if (info[4] != 0.0) return fail("kb_solve (PCG): grid barrier timed out");
  h->pcg_info.iterations = (int32_t)info[0];
  h->pcg_info.residual = info[1];
  h->pcg_info.d0 = info[2];
  h->pcg_residual = info[1];  // _residual = 0.5 dn (linear_solver_pcg.hpp:127)
  *ok = info[3] != 0.0 ? 1 : 0;
  return 0;
}

int kb_set_linear_solver(kb_handle* h, int32_t kind, const kb_pcg_options* pcg) {
  if (!h) return fail("kb_set_linear_solver: null");
  if (kind != KB_SOLVER_SCHUR && kind != KB_SOLVER_PCG && kind != KB_SOLVER_PCG_SCHUR)
    return fail("kb_set_linear_solver: unknown solver");
  if (kind == KB_SOLVER_PCG && sharded(h)) return fail("kb_set_linear_solver: PCG is not available on a sharded handle");
  h->solver_kind = kind;
  h->pcg = pcg ? *pcg : kb_pcg_options{1e-6, -1, 1};
  h->pcg_residual = -1.0;
  return 0;
}

int kb_pcg_init(kb_handle* h) {
  if (!h) return fail("kb_pcg_init: null");
  h->pcg_residual = -1.0;
  return 0;
}

int kb_get_pcg_info(kb_handle* h, kb_pcg_info* info) {
  if (!h || !info) return fail("kb_get_pcg_info: null");
  *info = h->pcg_info;
  return 0;
}

int kb_solve(kb_handle* h, double* dx_out, int* ok) {
  if (!h || !ok) return fail("kb_solve: null");
  KB_HIP(hipSetDevice(h->device));
  unprepare(h);
  if (h->solver_kind == KB_SOLVER_PCG) {
    if (h->use_cond) return fail("kb_solve (PCG): a diagonal conditioner is not supported, use a constant one");
    if (run_pcg(h, ok)) return -1;
    if (*ok && dx_out)
      KB_HIP(hipMemcpyAsync(dx_out, h->d.dx, sizeof(double) * h->ncols, hipMemcpyDeviceToHost, h->stream));
    KB_HIP(hipStreamSynchronize(h->stream));
    return 0;
  }
  const int one = 1;
  KB_HIP(hipMemcpyAsync(&h->d.ctrl->solve_ok, &one, sizeof(int), hipMemcpyHostToDevice, h->stream));
  struct CondScope {  // the diagonal conditioner (kb_set_conditioner) enters this solve's frame and camera blocks
    kb_handle* h;
    CondScope(kb_handle* hh) : h(hh) { h->d.cond2 = h->use_cond ? h->cond2 : nullptr; }
    ~CondScope() { h->d.cond2 = nullptr; }
  } cs(h);
  if (launch_schur(h, 0)) return -1;
  if (launch_colsum(h, 0)) return -1;
  // k_solve folds the frame-block failure count and the LDL^T of S (or PCG on S) into ctrl->solve_ok
  const bool pcs = h->solver_kind == KB_SOLVER_PCG_SCHUR;
  if (pcs) {
    if (ensure_pcg(h)) return -1;
    h->d.pcs_cb = h->pcg_cb;
    h->d.pcs_tol = h->pcg.tolerance;
    h->d.pcs_prev = h->pcg_residual;
    h->d.pcs_maxit = h->pcg.max_iterations < 0 ? h->C : h->pcg.max_iterations;
    h->d.pcs_abs = h->pcg.absolute_tolerance ? 1 : 0;
    h->d.pcs_info = h->pcg_buf + (size_t)h->F * (h->C + 1) + h->F + 8;  // after the full-system PCG's info [8]
  }
  const int rs = launch_solve(h, 0, 0);
  h->d.pcs_cb = nullptr;
  if (rs) return -1;
  int okd = 0;
  KB_HIP(hipMemcpyAsync(&okd, &h->d.ctrl->solve_ok, sizeof(int), hipMemcpyDeviceToHost, h->stream));
  double pinfo[4] = {0, 0, 0, 0};
  if (pcs) KB_HIP(hipMemcpyAsync(pinfo, h->d.pcs_info, sizeof(pinfo), hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  if (pcs && okd && pinfo[3] != 0.0) {
    // only a completed solve sets _residual (linear_solver_pcg.hpp:127): a failed one (singular DV block,
    // non-positive curvature) leaves the previous solve's values for the next absolute-tolerance d0
    h->pcg_info.iterations = (int32_t)pinfo[0];
    h->pcg_info.residual = pinfo[1];
    h->pcg_info.d0 = pinfo[2];
    h->pcg_residual = pinfo[1];  // _residual = 0.5 dn (linear_solver_pcg.hpp:127)
  }
  *ok = okd;
  if (!okd) return 0;
  if (launch_backsub(h, 0, 0, 0)) return -1;
  if (dx_out) KB_HIP(hipMemcpyAsync(dx_out, h->d.dx, sizeof(double) * h->ncols, hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kb_get_rhs(kb_handle* h, double* rhs_out) {
  if (!h || !rhs_out) return fail("kb_get_rhs: null");
  KB_HIP(hipSetDevice(h->device));
  KB_HIP(hipMemcpyAsync(rhs_out, h->d.gc, sizeof(double) * h->C, hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipMemcpyAsync(rhs_out + h->C, h->d.gf, sizeof(double) * 6 * h->F, hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kb_apply_update(kb_handle* h, const double* dx, double* deltaX_out) {
  if (!h) return fail("kb_apply_update: null");
  KB_HIP(hipSetDevice(h->device));
  unprepare(h);
  std::vector<double> hx;
  if (dx) {
    KB_HIP(hipMemcpyAsync(h->d.dx, dx, sizeof(double) * h->ncols, hipMemcpyHostToDevice, h->stream));
  } else {
    hx.resize(h->ncols);
    KB_HIP(hipMemcpyAsync(hx.data(), h->d.dx, sizeof(double) * h->ncols, hipMemcpyDeviceToHost, h->stream));
  }
  const int n = std::max(h->F, h->N * KB_MAX_INTR);
  hipLaunchKernelGGL(k_update_all, dim3((n + 255) / 256), dim3(256), 0, h->stream, h->d);
  KB_HIP(hipGetLastError());
  if (set_cur(h, 1 - h->cur)) return -1;
  KB_HIP(hipStreamSynchronize(h->stream));
  if (deltaX_out) {
    const double* p = dx ? dx : hx.data();
    double m = 0.0;
    for (int q = 0; q < h->ncols; ++q) m = std::max(m, std::fabs(p[q]));
    *deltaX_out = m;
  }
  return 0;
}

int kb_revert(kb_handle* h) {
  if (!h) return fail("kb_revert: null");
  KB_HIP(hipSetDevice(h->device));
  unprepare(h);
  if (set_cur(h, 1 - h->cur)) return -1;
  KB_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

// ---------------------------------------------------------------- marginal SVD solver (calibration::LinearSolver)
// the k_marg instance for C: full-storage Omega while it fits in LDS, packed upper beyond
using MargKernel = void (*)(KbDev, KbMarg, int);
static MargKernel marg_kernel(int C) { return marg_full(C) ? k_marg<true> : k_marg<false>; }
static const void* marg_fn(int C) { return (const void*)marg_kernel(C); }

// warm-started Jacobi sweeps (k_marg) unless KB_MARG_COLD is set (A/B runs: every call from V = I, as Eigen::JacobiSVD)
static int marg_warm() {
  static const int w = std::getenv("KB_MARG_COLD") ? 0 : 1;
  return w;
}

static void marg_info(const double* inf, kb_marginal_info* info) {
  if (!info) return;
  info->rank = (int32_t)inf[0];
  info->sweeps = (int32_t)inf[1];
  info->tolerance = inf[2];
  info->sv_gap = inf[3];
  info->sv_log2_sum = inf[4];
}

// the marginal camera solve (write_dx) or analyzeMarginal (unscaled SVD only) enqueued on the stream: the frame blocks
// of the last build eliminated at lambda = 0, the column sums, k_marg, and the copies of info [8] / sv / V out (the
// caller syncs)
static int enqueue_marginal(kb_handle* h, const kb_marginal_options* o, int write_dx, double* inf, double* sv_out,
                            double* V_out) {
  if (h->C > kMargMaxC) return fail("marginal solver: camera block C > 112 is not supported");
  if (sharded(h)) return fail("marginal solver: not available on a sharded handle");
  const int C = h->C;
  const size_t mstride = (size_t)C * C + C + 8;
  if (!h->marg_buf && h->alloc(&h->marg_buf, 2 * mstride)) return -1;
  KbMarg m{};
  m.scaling = o->column_scaling ? 1 : 0;
  m.write_dx = write_dx;
  m.warm = marg_warm();
  m.norm_tol = std::sqrt(2.0 * (double)h->NC * o->eps_norm);  // rows of J: 2 per corner
  m.eps_svd = o->eps_svd;
  m.svd_tol = o->svd_tol;
  m.V = h->marg_buf + (write_dx ? 0 : mstride);  // solve and analyzeMarginal keep their own warm-start V
  m.sv = m.V + (size_t)C * C;
  m.info = m.sv + C;
  const double lam_saved = h->d.host_lambda;
  h->d.host_lambda = 0.0;
  int rc = launch_schur(h, 0);
  if (!rc) rc = launch_colsum(h, 0);
  h->d.host_lambda = lam_saved;
  if (rc) return rc;
  bool stage_v0;
  const size_t lds = sizeof(double) * (size_t)marg_lds_doubles(C, stage_v0);
  KB_HIP(hipFuncSetAttribute(marg_fn(C), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(marg_kernel(C), dim3(1), dim3(marg_block(C)), lds, h->stream, h->d, m, 0);
  KB_HIP(hipGetLastError());
  KB_HIP(hipMemcpyAsync(inf, m.info, sizeof(double) * 8, hipMemcpyDeviceToHost, h->stream));
  if (sv_out) KB_HIP(hipMemcpyAsync(sv_out, m.sv, sizeof(double) * C, hipMemcpyDeviceToHost, h->stream));
  if (V_out) KB_HIP(hipMemcpyAsync(V_out, m.V, sizeof(double) * C * C, hipMemcpyDeviceToHost, h->stream));
  return 0;
}

static int run_marginal(kb_handle* h, const kb_marginal_options* o, int write_dx, kb_marginal_info* info,
                        double* sv_out, double* V_out) {
  double inf[8];
  if (enqueue_marginal(h, o, write_dx, inf, sv_out, V_out)) return -1;
  KB_HIP(hipStreamSynchronize(h->stream));
  marg_info(inf, info);
  return 0;
}

int kb_solve_marginal(kb_handle* h, const kb_marginal_options* opts, double* dx_out, int* ok, kb_marginal_info* info,
                      double* sv_out, double* V_out) {
  if (!h || !opts || !ok) return fail("kb_solve_marginal: null");
  KB_HIP(hipSetDevice(h->device));
  unprepare(h);
  const int one = 1;
  KB_HIP(hipMemcpyAsync(&h->d.ctrl->solve_ok, &one, sizeof(int), hipMemcpyHostToDevice, h->stream));
  if (run_marginal(h, opts, 1, info, sv_out, V_out)) return -1;
  int okd = 0;
  KB_HIP(hipMemcpyAsync(&okd, &h->d.ctrl->solve_ok, sizeof(int), hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  *ok = okd;
  if (!okd) return 0;
  if (launch_backsub(h, 0, 0, 0)) return -1;  // frame steps from the lambda = 0 blocks k_schur left
  if (dx_out) KB_HIP(hipMemcpyAsync(dx_out, h->d.dx, sizeof(double) * h->ncols, hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kb_analyze_marginal(kb_handle* h, const kb_marginal_options* opts, kb_marginal_info* info, double* sv_out,
                        double* V_out) {
  if (!h || !opts) return fail("kb_analyze_marginal: null");
  KB_HIP(hipSetDevice(h->device));
  kb_marginal_options un = *opts;
  un.column_scaling = 0;
  return run_marginal(h, &un, 0, info, sv_out, V_out);
}

int kb_get_normal_blocks(kb_handle* h, double* Hff, double* Hfc, double* gf, double* Hcc, double* gc, double* cost) {
  if (!h) return fail("null handle");
  if (!h->sys_valid) return fail("kb_get_normal_blocks: no intact system (call kb_build first; the optimizer loops "
                                 "do not leave the per-call blocks)");
  KB_HIP(hipSetDevice(h->device));
  if (Hff) KB_HIP(hipMemcpyAsync(Hff, h->d.Hff, sizeof(double) * 36 * h->F, hipMemcpyDeviceToHost, h->stream));
  if (Hfc) KB_HIP(hipMemcpyAsync(Hfc, h->d.Hfc, sizeof(double) * 6 * h->C * h->F, hipMemcpyDeviceToHost, h->stream));
  if (gf) KB_HIP(hipMemcpyAsync(gf, h->d.gf, sizeof(double) * 6 * h->F, hipMemcpyDeviceToHost, h->stream));
  if (Hcc) KB_HIP(hipMemcpyAsync(Hcc, h->d.Hcc, sizeof(double) * h->C * h->C, hipMemcpyDeviceToHost, h->stream));
  if (gc) KB_HIP(hipMemcpyAsync(gc, h->d.gc, sizeof(double) * h->C, hipMemcpyDeviceToHost, h->stream));
  if (cost) KB_HIP(hipMemcpyAsync(cost, h->d.cost_build, sizeof(double), hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kb_reprojection_error_stats(kb_handle* h, double* out) {
  if (!h || !out) return fail("kb_reprojection_error_stats: null");
  if (!h->uploaded) return fail("kb_reprojection_error_stats: no observations");
  KB_HIP(hipSetDevice(h->device));
  const int N = h->N, V = h->V;
  double* buf = nullptr;  // vpart [V][3] | pass-one sums [N][3] (+ [N][3] over ranks) | pass-two sums (same)
  const size_t nv = 3 * (size_t)std::max(V, 1), ns = 3 * (size_t)N;
  KB_HIP(hipMalloc(&buf, sizeof(double) * (nv + 4 * ns)));
  double *vpart = buf, *s1 = buf + nv, *s1r = s1 + ns, *s2 = s1r + ns, *s2r = s2 + ns;
  auto pass = [&](const double* sums, double* o, double* orr) -> int {
    hipLaunchKernelGGL(k_rstats, dim3((V + 3) / 4), dim3(256), 0, h->stream, h->d, sums, vpart);
    hipLaunchKernelGGL(k_rstats_red, dim3(N), dim3(256), 0, h->stream, h->d, vpart, o);
    KB_HIP(hipGetLastError());
    if (!sharded(h)) return hipMemcpyAsync(orr, o, sizeof(double) * ns, hipMemcpyDeviceToDevice, h->stream) == hipSuccess ? 0 : -1;
    return coll_allreduce(h, o, orr, ns);  // the ranks' frames: counts and sums over all of them
  };
  std::vector<double> a(ns), b(ns);
  int rc = V > 0 ? pass(nullptr, s1, s1r) : 0;
  if (!rc && V > 0) rc = pass(s1r, s2, s2r);
  if (!rc && V > 0) {
    if (hipMemcpyAsync(a.data(), s1r, sizeof(double) * ns, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
        hipMemcpyAsync(b.data(), s2r, sizeof(double) * ns, hipMemcpyDeviceToHost, h->stream) != hipSuccess)
      rc = -1;
  }
  if (hipStreamSynchronize(h->stream) != hipSuccess) rc = -1;
  hipFree(buf);
  if (rc) return fail("kb_reprojection_error_stats: device pass failed");
  // per camera [n, mean (2), sample std (2, N - 1), "RMSE" = |sum e| / sqrt(n)] (CameraCalibrator.hpp:378-410)
  for (int c = 0; c < N; ++c) {
    const double n = V > 0 ? a[3 * c] : 0.0;
    double* o = out + 6 * c;
    o[0] = n;
    o[1] = n > 0 ? a[3 * c + 1] / n : 0.0;
    o[2] = n > 0 ? a[3 * c + 2] / n : 0.0;
    o[3] = n > 1 ? std::sqrt(b[3 * c + 1] / (n - 1.0)) : 0.0;
    o[4] = n > 1 ? std::sqrt(b[3 * c + 2] / (n - 1.0)) : 0.0;
    o[5] = n > 0 ? std::sqrt(a[3 * c + 1] * a[3 * c + 1] + a[3 * c + 2] * a[3 * c + 2]) / std::sqrt(n) : 0.0;
  }
  return 0;
}

int kb_rhs_jtj_rhs(kb_handle* h, double* out) {
  if (!h || !out) return fail("kb_rhs_jtj_rhs: null");
  if (!h->uploaded) return fail("kb_rhs_jtj_rhs: no observations");
  if (!h->sys_valid) return fail("kb_rhs_jtj_rhs: no intact system (call kb_build first; the optimizer loops do "
                                 "not leave the per-call blocks)");
  if (sharded(h)) return fail("kb_rhs_jtj_rhs: per-call quantity of an unsharded handle");
  KB_HIP(hipSetDevice(h->device));
  if (h->rjr_F < (size_t)h->F + 1) {  // (re)sized for the current frame count (kb_append_frames grows it)
    if (regrow(h, &h->rjr, (size_t)h->F + 1, 0)) return -1;
    h->rjr_F = (size_t)h->F + 1;
  }
  hipLaunchKernelGGL(k_rjr_frames, dim3((h->F + 3) / 4), dim3(256), 0, h->stream, h->d, h->rjr);
  hipLaunchKernelGGL(k_rjr_final, dim3(1), dim3(256), 0, h->stream, h->d, h->rjr, h->rjr + h->F);
  KB_HIP(hipGetLastError());
  KB_HIP(hipMemcpyAsync(out, h->rjr + h->F, sizeof(double), hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

// ---------------------------------------------------------------- device-resident loop
// One optimizer pass: build (+ fused Schur) | [schur, LM passes that keep the system] | colsum [all-reduce] |
// solve (+ candidate camera chains) | backsub + cost, its last block: reduce, accept/revert, next prelude
// ([all-reduce + k_policy] when sharded).  Every kernel early-exits once ctrl->done is set.
// GN fused passes: [frame steps of the previous solve + build at that candidate] | colsum | [previous pass's
// end + solve]; the back-substitution and cost kernels drop out (the build's chi^2 is the candidate's cost).
// The launches see a KbDev with gn_fused set for the scope.
struct GnFusedScope {
  kb_handle* h;
  KbDev saved;
  GnFusedScope(kb_handle* hh, bool on) : h(hh), saved(hh->d) {
    if (on) {
      h->d.gn_fused = 1;
      h->d.fold = 0;
      h->d.xexp = h->xexp && h->nranks <= kXMaxRanks && (!sharded(h) || h->ximg_part) ? 1 : 0;
      h->d.ximg = sharded(h) ? h->ximg_part : h->d.simg;
    }
  }
  ~GnFusedScope() { h->d = saved; }
};

static bool gn_fused(const kb_handle* h, int policy) { return policy == 1 && h->gn_fuse; }

// ev0 / ev1 (optional): HIP events recorded around the build kernel (kb_build_kernel_stats)
static int enqueue_marg_pass(kb_handle* h);

static int enqueue_pass(kb_handle* h, int policy, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr) {
  if (policy == kPolicyMarginal) return enqueue_marg_pass(h);
  KbDev& d = h->d;
  auto build = [&]() -> int {
    if (ev0) KB_HIP(hipEventRecord(ev0, h->stream));
    if (launch_build(h, 1, 1)) return -1;
    if (ev1) KB_HIP(hipEventRecord(ev1, h->stream));
    return 0;
  };
  if (gn_fused(h, policy)) {
    GnFusedScope scope(h, true);
    const bool from_rows = h->d.Wp <= 2048;
    if (build() || launch_colsum(h, 1, !from_rows) || launch_solve(h, 1, 1, from_rows)) return -1;
    return 0;
  }
  if (build()) return -1;
  if (policy == 0 && launch_schur(h, 1)) return -1;  // LM passes that keep the system (lambda change)
  // small partial row: k_solve sums the stage-1 rows while staging (one launch less; sharded, the rows are
  // all-reduced as they are); otherwise k_colfin finishes the rows in parallel (then one row is all-reduced)
  const bool from_rows = h->d.Wp <= 2048;
  if (launch_colsum(h, 1, !from_rows)) return -1;
  if (launch_solve(h, 1, 1, from_rows)) return -1;
  if (launch_backsub(h, 1, 1, 1)) return -1;
  // the pass end (accept / revert, next prelude): one block (k_post); sharded, the per-frame step rows of every
  // rank are all-gathered first and every rank reduces all of them in rank order
  if (sharded(h) && coll_allgather(h, d.bpart, h->bpart_all, 4 * (size_t)h->F_max)) return -1;
  if (!d.fold) {
    hipLaunchKernelGGL(k_post, dim3(1), dim3(256), 0, h->stream, d, 1);
    KB_HIP(hipGetLastError());
  }
  return 0;
}

// device copy of the loop-visible handle state (both state buffers, the camera chains of both slots, the control block)
// and its restore: queries and warm-up launches leave the handle as they found it
struct Snapshot {
  kb_handle* h;
  double* buf = nullptr;
  int cur0 = 0;
  bool taken = false;
  explicit Snapshot(kb_handle* hh) : h(hh) {}
  Snapshot(const Snapshot&) = delete;
  Snapshot& operator=(const Snapshot&) = delete;
  int copy(bool restore) {
    KbDev& dv = h->d;
    const size_t sz[4] = {2 * (size_t)dv.S * 8, 2 * 12 * (size_t)h->N * 8, 2 * 36 * (size_t)h->N * h->N * 8,
                          sizeof(KbCtrl)};
    void* bufs[4] = {dv.state, dv.camL, dv.camK, dv.ctrl};
    if (!buf) {
      size_t tot = 0;
      for (size_t z : sz) tot += (z + 7) & ~size_t(7);
      KB_HIP(hipMalloc(&buf, tot));
    }
    char* c = (char*)buf;
    for (int q = 0; q < 4; ++q) {
      KB_HIP(hipMemcpyAsync(restore ? bufs[q] : c, restore ? c : bufs[q], sz[q], hipMemcpyDeviceToDevice, h->stream));
      c += (sz[q] + 7) & ~size_t(7);
    }
    return 0;
  }
  int take() {
    cur0 = h->cur;
    if (copy(false)) return -1;
    taken = true;
    return 0;
  }
  int restore() {
    if (copy(true)) return -1;
    h->cur = cur0;
    return 0;
  }
  ~Snapshot() {
    if (taken) {
      copy(true);
      hipStreamSynchronize(h->stream);
      h->cur = cur0;
    }
    if (buf) hipFree(buf);
  }
};

static int ensure_trace(kb_handle* h, int cap) {
  if (h->trace_cap >= cap) return 0;
  if (h->trace) hipFree(h->trace);
  h->trace = nullptr;
  KB_HIP(hipMalloc(&h->trace, sizeof(double) * 4 * cap));
  h->trace_cap = cap;
  h->d.trace = h->trace;
  h->d.trace_cap = cap;
  drop_graphs(h);  // captured kernel args hold the old pointer
  return 0;
}

static int capture(kb_handle* h, int policy, int passes, hipGraphExec_t* out) {
  hipGraph_t g = nullptr;
  KB_HIP(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
  int rc = 0;
  for (int i = 0; i < passes && !rc; ++i) rc = enqueue_pass(h, policy);
  hipError_t e = hipStreamEndCapture(h->stream, &g);
  if (rc) return rc;
  if (e != hipSuccess) return fail(std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
  KB_HIP(hipGraphInstantiate(out, g, nullptr, nullptr, 0));
  KB_HIP(hipGraphDestroy(g));
  KB_HIP(hipGraphUpload(*out, h->stream));  // the first launch then costs what every later one does
  return 0;
}

static int ensure_graph(kb_handle* h, int policy) {
  if (h->graphs[kGraphPasses] && h->graph_policy == policy) return 0;
  drop_graphs(h);
  if (capture(h, policy, kGraphPasses, &h->graphs[kGraphPasses])) return -1;
  h->graph_policy = policy;
  return 0;
}

// the graph of k passes (k <= kGraphPasses) of the current graph policy, captured on first use
static int graph_of(kb_handle* h, int k, hipGraphExec_t* out) {
  if (!h->graphs[k] && capture(h, h->graph_policy, k, &h->graphs[k])) return -1;
  *out = h->graphs[k];
  return 0;
}

// captured graphs for this policy; RCCL calls are captured too when sharded.  If capturing them fails on this
// stack, the handle falls back to eager passes for good (same kernels, same results).
static bool graph_ok(kb_handle* h, int policy) {
  if (h->graph_failed || h->lg) return false;  // the in-process group's collectives meet on the host: eager
  if (ensure_graph(h, policy) == 0) return true;
  if (!h->comm) return false;  // caller reports the error through kb_last_error on the eager path as well
  hipGetLastError();
  drop_graphs(h);
  h->graph_failed = true;
  return false;
}

// launch n passes: whole kGraphPasses graphs, then one graph of the n % kGraphPasses remaining passes, so every
// pass runs inside a multi-pass graph whatever n is (or eager passes when not graphed)
static int launch_passes(kb_handle* h, int policy, int n, bool graph) {
  if (!graph) {
    for (int i = 0; i < n; ++i)
      if (enqueue_pass(h, policy)) return -1;
    return 0;
  }
  const int rem = n % kGraphPasses;
  hipGraphExec_t gr = nullptr;
  if (rem && graph_of(h, rem, &gr)) return -1;  // captured before the launches (capture uses the stream)
  for (int i = 0; i + kGraphPasses <= n; i += kGraphPasses) KB_HIP(hipGraphLaunch(h->graphs[kGraphPasses], h->stream));
  if (rem) KB_HIP(hipGraphLaunch(gr, h->stream));
  return 0;
}

// the last pass's pending end (accept / revert) when the loop stops: no-op if nothing is pending
static int finish_pass(kb_handle* h, int policy) {
  if (gn_fused(h, policy)) {  // the last solve's step: back-substitution + cost, then its end as usual
    GnFusedScope scope(h, true);
    if (launch_backsub(h, 1, 1, 1)) return -1;
    if (sharded(h) && coll_allgather(h, h->d.bpart, h->bpart_all, 4 * (size_t)h->F_max)) return -1;
  }
  hipLaunchKernelGGL(k_post, dim3(1), dim3(256), 0, h->stream, h->d, 1);
  KB_HIP(hipGetLastError());
  return 0;
}

// a loop start on a rank of a direct all-reduce group: the ranks agree (a sum over the collective, so every rank
// runs it whatever its own outcome) whether any of them saw a k_xar wait time out since the last loop start; if one
// did, every rank leaves the direct path for the collective for good.  The flag counters of the ranks may have
// drifted apart in the failed batch (a failing rank skips its remaining passes), so the direct path is not resumed.
static void xar_uninstall(kb_handle* h);
static int xar_agree(kb_handle* h) {
  if (!sharded(h) || !h->d.xar) return 0;
  const double mine = h->xar_failed ? 1.0 : 0.0;
  double sum = 0.0;
  KB_HIP(hipMemcpyAsync(h->xar_agree_buf, &mine, sizeof(double), hipMemcpyHostToDevice, h->stream));
  if (coll_allreduce(h, h->xar_agree_buf, h->xar_agree_buf + 1, 1)) return -1;
  KB_HIP(hipMemcpyAsync(&sum, h->xar_agree_buf + 1, sizeof(double), hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  if (sum > 0.0) xar_uninstall(h);
  h->xar_failed = false;
  return 0;
}

static int loop_start(kb_handle* h, const KbOpts& o) {
  // evaluateError on the start state (Optimizer2.cpp:192-196), optimizationStarting, first prelude
  if (xar_agree(h)) return -1;
  unprepare(h);
  h->sys_valid = false;  // the loop's passes overwrite g_c (and skip the frame-block stores when GN fused)
  if (launch_cost(h, 0)) return -1;
  if (allreduce_red(h)) return -1;
  hipLaunchKernelGGL(k_pol_init, dim3(1), dim3(1), 0, h->stream, h->d, o);
  hipLaunchKernelGGL(k_pre, dim3(1), dim3(256), 0, h->stream, h->d, 1);
  KB_HIP(hipGetLastError());
  return 0;
}

int kb_optimize(kb_handle* h, const kb_optimizer_options* opts, kb_solution* out) {
  if (!h || !opts || !out) return fail("kb_optimize: null");
  if (!h->uploaded) return fail("kb_optimize: no observations");
  if (opts->policy != 0 && opts->policy != 1) return fail("kb_optimize: unknown policy");
  KB_HIP(hipSetDevice(h->device));
  const int max_passes = 2 * opts->max_iterations + 1;
  if (ensure_trace(h, max_passes + 1)) return -1;
  KbOpts o{opts->policy, opts->max_iterations, opts->lambda_init, opts->convergence_dx, opts->convergence_dj};
  if (loop_start(h, o)) return -1;
  const bool graph = opts->use_graph != 0 && graph_ok(h, opts->policy);
  const int every = opts->sync_every > 0 ? opts->sync_every : 2 * kGraphPasses;
  KbCtrl ctrl{};
  int passes = 0;
  while (passes < max_passes) {
    const int n = std::min(every, max_passes - passes);
    if (launch_passes(h, opts->policy, n, graph)) return -1;
    passes += n;
    KB_HIP(hipMemcpyAsync(&ctrl, h->d.ctrl, sizeof(KbCtrl), hipMemcpyDeviceToHost, h->stream));
    KB_HIP(hipStreamSynchronize(h->stream));
    if (comm_check(h, ctrl)) return -1;
    if (ctrl.done) break;
  }
  if (finish_pass(h, opts->policy)) return -1;
  KB_HIP(hipMemcpy(&ctrl, h->d.ctrl, sizeof(KbCtrl), hipMemcpyDeviceToHost));
  if (comm_check(h, ctrl)) return -1;
  h->cur = ctrl.cur;
  out->J_start = ctrl.J_start;
  out->J_final = ctrl.p_J;
  out->dx_final = ctrl.deltaX;
  out->dj_final = ctrl.deltaJ;
  out->iterations = ctrl.iterations;
  out->failed_iterations = ctrl.failed_iterations;
  out->linear_solver_failure = ctrl.lin_fail;
  out->passes = ctrl.passes;
  out->graphed = graph ? 1 : 0;
  return 0;
}

// one pass of the device-resident IncrementalEstimator loop (Optimizer2 + GaussNewtonTrustRegionPolicy over
// calibration::LinearSolver, IncrementalEstimator.cpp:46-77, 373): build with the frame blocks eliminated at
// lambda = 0 (the policy's lambda), column sums, H_cc / g_c, the column-scaled truncated-SVD camera step (k_marg),
// the candidate camera design variables and chains (the end of the gated k_marg), the frame steps and the candidate's cost
// (k_backsub), the pass end (k_post: accept, convergence tests, next prelude).  Every kernel is gated on ctrl.
static int enqueue_marg_pass(kb_handle* h) {
  if (launch_build(h, 1, 1) || launch_colsum(h, 1, false)) return -1;
  // the two column-sum consumers (k_camexpand, k_marg) sum the kColsumRows stage-1 rows themselves, in k_colfin's
  // order: one launch less per pass
  KbDev dr = h->d;
  dr.psum = dr.part8;
  dr.psum_rows = kColsumRows;
  hipLaunchKernelGGL(k_camexpand, dim3(1), dim3(256), h->lds_camexp, h->stream, dr, 1);
  hipLaunchKernelGGL(marg_kernel(h->C), dim3(1), dim3(marg_block(h->C)), h->lds_marg, h->stream, dr, h->marg, 1);
  KB_HIP(hipGetLastError());
  if (launch_backsub(h, 1, 1, 1)) return -1;
  hipLaunchKernelGGL(k_post, dim3(1), dim3(256), 0, h->stream, h->d, 1);
  KB_HIP(hipGetLastError());
  return 0;
}

static int optimize_marginal(kb_handle* h, const kb_optimizer_options* opts, const kb_marginal_options* mopts,
                             kb_solution* out, kb_marginal_info* info, double* sv_out, double* V_out, bool analyze,
                             kb_marginal_info* ainfo, double* asv_out, double* aV_out) {
  if (!h || !opts || !mopts || !out) return fail("kb_optimize_marginal: null");
  if (!h->uploaded) return fail("kb_optimize_marginal: no observations");
  if (opts->policy != 1) return fail("kb_optimize_marginal: the IncrementalEstimator's policy is Gauss-Newton (1)");
  if (h->C > kMargMaxC) return fail("kb_optimize_marginal: camera block C > 112 is not supported");
  if (sharded(h)) return fail("kb_optimize_marginal: not available on a sharded handle");
  KB_HIP(hipSetDevice(h->device));
  const int C = h->C;
  if (!h->marg_buf && h->alloc(&h->marg_buf, 2 * ((size_t)C * C + C + 8))) return -1;
  KbMarg m{};
  m.scaling = mopts->column_scaling ? 1 : 0;
  m.write_dx = 1;
  m.warm = marg_warm();
  m.norm_tol = std::sqrt(2.0 * (double)h->NC * mopts->eps_norm);
  m.eps_svd = mopts->eps_svd;
  m.svd_tol = mopts->svd_tol;
  m.V = h->marg_buf;
  m.sv = m.V + (size_t)C * C;
  m.info = m.sv + C;
  bool stage_v0;
  h->lds_marg = sizeof(double) * (size_t)marg_lds_doubles(C, stage_v0);
  KB_HIP(hipFuncSetAttribute(marg_fn(C), hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_marg));
  // the captured passes hold the k_marg arguments: other options (or a grown problem: norm_tol) recapture them
  if (std::memcmp(&m, &h->marg, sizeof(KbMarg)) != 0) {
    if (h->graph_policy == kPolicyMarginal) drop_graphs(h);
    h->marg = m;
  }
  const int max_passes = 2 * opts->max_iterations + 1;
  if (ensure_trace(h, max_passes + 1)) return -1;
  KbOpts o{1, opts->max_iterations, 0.0, opts->convergence_dx, opts->convergence_dj};
  if (loop_start(h, o)) return -1;
  const bool graph = opts->use_graph != 0 && graph_ok(h, kPolicyMarginal);
  const int every = opts->sync_every > 0 ? opts->sync_every : 2 * kGraphPasses;
  KbCtrl ctrl{};
  int passes = 0;
  while (passes < max_passes) {
    const int n = std::min(every, max_passes - passes);
    if (launch_passes(h, kPolicyMarginal, n, graph)) return -1;
    passes += n;
    KB_HIP(hipMemcpyAsync(&ctrl, h->d.ctrl, sizeof(KbCtrl), hipMemcpyDeviceToHost, h->stream));
    KB_HIP(hipStreamSynchronize(h->stream));
    if (comm_check(h, ctrl)) return -1;
    if (ctrl.done) break;
  }
  if (finish_pass(h, kPolicyMarginal)) return -1;
  double inf[8], ainf[8];
  KB_HIP(hipMemcpyAsync(&ctrl, h->d.ctrl, sizeof(KbCtrl), hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipMemcpyAsync(inf, m.info, sizeof(inf), hipMemcpyDeviceToHost, h->stream));
  if (sv_out) KB_HIP(hipMemcpyAsync(sv_out, m.sv, sizeof(double) * C, hipMemcpyDeviceToHost, h->stream));
  if (V_out) KB_HIP(hipMemcpyAsync(V_out, m.V, sizeof(double) * C * C, hipMemcpyDeviceToHost, h->stream));
  if (analyze) {  // analyzeMarginal of the last built system, in the same stream sync (IncrementalEstimator.cpp:400)
    kb_marginal_options un = *mopts;
    un.column_scaling = 0;
    if (enqueue_marginal(h, &un, 0, ainf, asv_out, aV_out)) return -1;
  }
  KB_HIP(hipStreamSynchronize(h->stream));
  if (comm_check(h, ctrl)) return -1;
  if (analyze) marg_info(ainf, ainfo);
  h->cur = ctrl.cur;
  out->J_start = ctrl.J_start;
  out->J_final = ctrl.p_J;
  out->dx_final = ctrl.deltaX;
  out->dj_final = ctrl.deltaJ;
  out->iterations = ctrl.iterations;
  out->failed_iterations = ctrl.failed_iterations;
  out->linear_solver_failure = ctrl.lin_fail;
  out->passes = ctrl.passes;
  out->graphed = graph ? 1 : 0;
  if (info) {
    info->rank = (int32_t)inf[0];
    info->sweeps = (int32_t)inf[1];
    info->tolerance = inf[2];
    info->sv_gap = inf[3];
    info->sv_log2_sum = inf[4];
  }
  return 0;
}

int kb_optimize_marginal(kb_handle* h, const kb_optimizer_options* opts, const kb_marginal_options* mopts,
                         kb_solution* out, kb_marginal_info* info, double* sv_out, double* V_out) {
  return optimize_marginal(h, opts, mopts, out, info, sv_out, V_out, false, nullptr, nullptr, nullptr);
}

int kb_optimize_marginal_analyze(kb_handle* h, const kb_optimizer_options* opts, const kb_marginal_options* mopts,
                                 kb_solution* out, kb_marginal_info* info, double* sv_out, double* V_out,
                                 kb_marginal_info* analyze_info, double* analyze_sv_out, double* analyze_V_out) {
  return optimize_marginal(h, opts, mopts, out, info, sv_out, V_out, true, analyze_info, analyze_sv_out,
                           analyze_V_out);
}

int kb_get_trace(kb_handle* h, double* trace, int32_t cap) {
  if (!h || !trace) return fail("kb_get_trace: null");
  KB_HIP(hipSetDevice(h->device));
  KbCtrl ctrl{};
  KB_HIP(hipMemcpy(&ctrl, h->d.ctrl, sizeof(KbCtrl), hipMemcpyDeviceToHost));
  const int n = std::min(cap, std::min(ctrl.n_trace, h->trace_cap));
  if (n > 0) KB_HIP(hipMemcpy(trace, h->trace, sizeof(double) * 4 * n, hipMemcpyDeviceToHost));
  return n;
}

// `passes` GN passes (+ the loop's end when `with_end`) captured as one graph
static int capture_gn(kb_handle* h, int passes, bool with_end, hipGraphExec_t* out) {
  hipGraph_t g = nullptr;
  KB_HIP(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
  int rc = 0;
  for (int i = 0; i < passes && !rc; ++i) rc = enqueue_pass(h, 1);
  if (!rc && with_end) rc = finish_pass(h, 1);
  const hipError_t e = hipStreamEndCapture(h->stream, &g);
  if (rc) {
    if (g) hipGraphDestroy(g);
    return rc;
  }
  if (e != hipSuccess) return fail(std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
  const hipError_t ei = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
  hipGraphDestroy(g);
  if (ei != hipSuccess) return fail(std::string("hipGraphInstantiate: ") + hipGetErrorString(ei));
  KB_HIP(hipGraphUpload(*out, h->stream));
  return 0;
}

int kb_gn_prepare(kb_handle* h, int32_t n_iter) {
  if (!h || n_iter < 0) return fail("kb_gn_prepare: bad args");
  if (!h->uploaded) return fail("kb_gn_prepare: no observations");
  KB_HIP(hipSetDevice(h->device));
  if (ensure_trace(h, 64)) return -1;
  // GN, convergence tests disabled (thresholds -1 keep (dX > eps && |dJ| > eps) true)
  KbOpts o{1, 0x3fffffff, 0.0, -1.0, -1.0};
  if (xar_agree(h)) return -1;  // before the captures (leaving the direct path drops the graphs)
  h->gn_graph = graph_ok(h, 1);
  if (h->gn_graph) {
    // up to kGnOneGraph passes run as one graph with the loop's end (the last step's back-substitution and k_post)
    // captured behind them: no graph-to-graph gap and no eager launch inside the timed region.  Longer runs launch
    // whole kGnOneGraph-pass graphs first and the last 1..kGnOneGraph passes with the end as the tail graph.
    const int t = n_iter <= kGnOneGraph ? n_iter : (n_iter % kGnOneGraph ? n_iter % kGnOneGraph : kGnOneGraph);
    if (n_iter > t && !h->gn_big && capture_gn(h, kGnOneGraph, false, &h->gn_big)) return -1;
    if (h->gn_tail_n != t) {
      if (h->gn_tail) hipGraphExecDestroy(h->gn_tail);
      h->gn_tail = nullptr;
      h->gn_tail_n = -1;
      if (capture_gn(h, t, true, &h->gn_tail)) return -1;
      h->gn_tail_n = t;
    }
    h->gn_head = n_iter - t;
    // every graph the timed launch will use runs once here, from a snapshot that is restored afterwards: a graph's
    // first launch costs more than the later ones (measured ~0.2 ms per kb_gn_launch at configs[3] when the 8-pass graph
    // was first launched inside it), and that is set-up, not pass time.  Sharded: every rank prepares the same n_iter,
    // so the captured collectives of these launches are matched across the ranks.
    Snapshot snap(h);
    if (snap.take() || loop_start(h, o)) return -1;
    if (h->gn_head > 0) KB_HIP(hipGraphLaunch(h->gn_big, h->stream));
    KB_HIP(hipGraphLaunch(h->gn_tail, h->stream));
    if (snap.restore()) return -1;
    KB_HIP(hipStreamSynchronize(h->stream));
    snap.taken = false;
  }
  if (loop_start(h, o)) return -1;
  KB_HIP(hipStreamSynchronize(h->stream));
  h->gn_prepared = n_iter;
  return h->gn_graph ? 1 : 0;
}

int kb_gn_launch(kb_handle* h, int32_t n_iter, double* seconds) {
  if (!h || n_iter < 0) return fail("kb_gn_launch: bad args");
  if (h->gn_prepared != n_iter) return fail("kb_gn_launch: not prepared for this pass count (kb_gn_prepare)");
  h->gn_prepared = -1;
  KB_HIP(hipSetDevice(h->device));
  const bool graph = h->gn_graph;
  if (graph && (!h->gn_tail || h->gn_head + h->gn_tail_n != n_iter))
    return fail("kb_gn_launch: the prepared graphs do not cover this pass count");
  // KB_LAUNCH_DIAG=1 (diagnostics only): HIP events around the launches, and the host time to return from the
  // launches and from the sync, printed to stderr
  static const bool diag = std::getenv("KB_LAUNCH_DIAG") != nullptr;
  hipEvent_t de[2] = {nullptr, nullptr};
  if (diag) {
    KB_HIP(hipEventCreate(&de[0]));
    KB_HIP(hipEventCreate(&de[1]));
    KB_HIP(hipEventRecord(de[0], h->stream));
  }
  const auto t0 = std::chrono::steady_clock::now();
  if (graph) {
    for (int i = 0; i < h->gn_head; i += kGnOneGraph) KB_HIP(hipGraphLaunch(h->gn_big, h->stream));
    KB_HIP(hipGraphLaunch(h->gn_tail, h->stream));
  } else {
    if (launch_passes(h, 1, n_iter, false)) return -1;
    if (finish_pass(h, 1)) return -1;
  }
  const auto tl = std::chrono::steady_clock::now();
  if (diag) KB_HIP(hipEventRecord(de[1], h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  const auto t1 = std::chrono::steady_clock::now();
  if (diag) {
    float ms = 0.f;
    hipEventElapsedTime(&ms, de[0], de[1]);
    std::fprintf(stderr, "kb_gn_launch n=%d graph=%d host_launch_us=%.1f host_total_us=%.1f dev_span_us=%.1f\n", n_iter,
                 graph ? 1 : 0, 1e6 * std::chrono::duration<double>(tl - t0).count(),
                 1e6 * std::chrono::duration<double>(t1 - t0).count(), 1e3 * ms);
    hipEventDestroy(de[0]);
    hipEventDestroy(de[1]);
  }
  if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
  KbCtrl ctrl{};
  KB_HIP(hipMemcpy(&ctrl, h->d.ctrl, sizeof(KbCtrl), hipMemcpyDeviceToHost));
  h->cur = ctrl.cur;
  if (comm_check(h, ctrl)) return -1;
  if (ctrl.iterations != n_iter) return fail("kb_gn_launch: linear solver failures during the timed passes");
  return 0;
}

int kb_run_gn_iterations(kb_handle* h, int32_t n_iter, double* seconds) {
  if (kb_gn_prepare(h, n_iter) < 0) return -1;
  return kb_gn_launch(h, n_iter, seconds);
}

// n Gauss-Newton passes from the current state, captured in one graph so that the passes run exactly as in the
// benchmarked graphs (eager launches if this stack cannot capture, or when sharded).  A query: the state buffers, camera
// chains and control block are saved first and restored at the end, so the handle is left as it was.
//   build_ms[r]: HIP events around pass r's build kernel (event nodes in the graph)
//   pass_ms[r]:  pass r from its build's start to the next pass's build start, from an s_memrealtime stamp the build
//                kernel's block 0 takes at entry (KbDev::pass_ts; 100 MHz), in a separate run of n + 1 passes without
//                event nodes, which would otherwise add their own gaps to every pass
static int timed_gn_passes(kb_handle* h, int n, std::vector<double>& pass_ms, std::vector<double>& build_ms) {
  if (ensure_trace(h, 64)) return -1;
  Snapshot snap(h);
  if (snap.take()) return -1;
  KbOpts o{1, 0x3fffffff, 0.0, -1.0, -1.0};
  std::vector<hipEvent_t> ev(2 * n, nullptr);
  struct EvGuard {
    std::vector<hipEvent_t>* ev;
    ~EvGuard() {
      for (auto& e : *ev)
        if (e) hipEventDestroy(e);
    }
  } evg{&ev};
  for (auto& e : ev) KB_HIP(hipEventCreate(&e));
  unsigned long long* ts = nullptr;
  KB_HIP(hipMalloc(&ts, sizeof(unsigned long long) * (kPassTsCap + 1)));
  struct TsGuard {
    unsigned long long* p;
    ~TsGuard() { hipFree(p); }
  } tsg{ts};
  // run = 0: build events, n passes; run = 1: pass stamps, n + 1 passes
  auto enqueue_run = [&](int run) -> int {
    if (run == 0) {
      for (int r = 0; r < n; ++r)
        if (enqueue_pass(h, 1, ev[2 * r], ev[2 * r + 1])) return -1;
      return 0;
    }
    KbDev keep = h->d;
    h->d.pass_ts = ts;
    int rc = 0;
    for (int r = 0; r <= n && !rc; ++r) rc = enqueue_pass(h, 1);
    h->d = keep;
    return rc;
  };
  std::vector<unsigned long long> hts(kPassTsCap + 1);
  auto read_run = [&](int run) -> bool {
    if (run == 0) {
      build_ms.assign(n, 0.0);
      for (int r = 0; r < n; ++r) {
        float b = 0.f;
        if (hipEventElapsedTime(&b, ev[2 * r], ev[2 * r + 1]) != hipSuccess || !(b > 0.f)) return false;
        build_ms[r] = b;
      }
      return true;
    }
    if (hipMemcpy(hts.data(), ts, sizeof(unsigned long long) * (n + 2), hipMemcpyDeviceToHost) != hipSuccess) return false;
    if (hts[0] < (unsigned long long)(n + 1)) return false;
    pass_ms.assign(n, 0.0);
    for (int r = 0; r < n; ++r) pass_ms[r] = 1e-5 * (double)(hts[r + 2] - hts[r + 1]);  // 100 MHz ticks -> ms
    return true;
  };
  for (int run = 0; run < 2; ++run) {
    if (run == 1) {
      if (snap.restore()) return -1;
      KB_HIP(hipMemsetAsync(ts, 0, sizeof(unsigned long long) * (kPassTsCap + 1), h->stream));
    }
    if (loop_start(h, o)) return -1;
    bool ok = false;
    if (!sharded(h) && hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal) == hipSuccess) {
      const int rc = enqueue_run(run);
      hipGraph_t g = nullptr;
      const hipError_t e = hipStreamEndCapture(h->stream, &g);
      hipGraphExec_t ge = nullptr;
      if (!rc && e == hipSuccess && g && hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) == hipSuccess) {
        // launched twice: the first launch of a graph costs more than the later ones (kb_gn_prepare)
        bool l = hipGraphLaunch(ge, h->stream) == hipSuccess;
        if (l && run == 1) {
          l = snap.restore() == 0 && hipMemsetAsync(ts, 0, sizeof(unsigned long long) * (kPassTsCap + 1), h->stream) ==
                                         hipSuccess && loop_start(h, o) == 0;
          l = l && hipGraphLaunch(ge, h->stream) == hipSuccess;
        }
        ok = l && hipStreamSynchronize(h->stream) == hipSuccess;
        hipGraphExecDestroy(ge);
      }
      if (g) hipGraphDestroy(g);
      if (ok) ok = read_run(run);  // graph-recorded events without timing data on this stack: eager instead
      if (!ok) hipGetLastError();
    }
    if (!ok) {
      if (snap.restore()) return -1;
      if (run == 1) KB_HIP(hipMemsetAsync(ts, 0, sizeof(unsigned long long) * (kPassTsCap + 1), h->stream));
      if (loop_start(h, o) || enqueue_run(run)) return -1;
      KB_HIP(hipStreamSynchronize(h->stream));
      if (!read_run(run)) return fail("timed_gn_passes: no device timing on this stack");
    }
    if (finish_pass(h, 1)) return -1;
    KB_HIP(hipStreamSynchronize(h->stream));
  }
  return 0;  // (the snapshot restores the handle)
}

int kb_gn_pass_times(kb_handle* h, int32_t n, double* pass_ms, double* build_ms) {
  if (!h || n < 1 || n + 1 > kPassTsCap) return fail("kb_gn_pass_times: bad args (1 <= n < 255)");
  if (!h->uploaded) return fail("kb_gn_pass_times: no observations");
  KB_HIP(hipSetDevice(h->device));
  std::vector<double> pm, bm;
  if (timed_gn_passes(h, n, pm, bm)) return -1;
  for (int r = 0; r < n; ++r) {
    if (pass_ms) pass_ms[r] = pm[r];
    if (build_ms) build_ms[r] = bm[r];
  }
  return 0;
}

int kb_build_kernel_stats(kb_handle* h, double* avg_ms, double* bytes_per_launch, double* flops_per_launch) {
  if (!h) return fail("null handle");
  if (!h->uploaded) return fail("kb_build_kernel_stats: no observations");
  KB_HIP(hipSetDevice(h->device));
  // Gauss-Newton passes from the current state with HIP events around each build kernel: the timed launches are the
  // build exactly as it runs inside the pass (frame steps of the previous solve applied)
  const int reps = 20, warm = 2;
  std::vector<double> pm, bm;
  if (timed_gn_passes(h, reps + warm, pm, bm)) return -1;
  double tot = 0.0;
  for (int r = warm; r < reps + warm; ++r) tot += bm[r];
  h->build_ms = tot / reps;
  if (avg_ms) *avg_ms = h->build_ms;
  // algorithmic bytes of one launch: observations (y 16 B + corner id 2 B per corner), view ranges (8 B per
  // frame x camera), state and camera chains read; the previous step (dx_c, A_f, b_f) read; g_f (and outside GN
  // fused passes H_ff, H_fc), back-substitution rows (A_f, b_f), candidate poses and the per-block partial rows
  // written.
  const double C = h->C, F = h->F;
  const double fblk = gn_fused(h, 1) ? 6.0 : 36.0 + 6.0 + 6.0 * C;
  const double bytes = 18.0 * h->NC + 8.0 * F * h->N + 8.0 * h->S + 8.0 * (12.0 * h->N + 36.0 * h->N * h->N) +
                       8.0 * (C + F * (6 * C + 6)) + 8.0 * F * fblk + 8.0 * F * (6 * C + 6 + 7) +
                       8.0 * h->d.nblk * h->d.Wr;
  if (bytes_per_launch) *bytes_per_launch = bytes;
  // algorithmic FP64 flops of one pass's build (SURVEY.md 8(d) "Algorithmic FLOPs"), not the executed (padded) MFMA
  // work, and only the terms this kernel performs: per corner ~150 (projection + Jacobian; the candidate's chi^2 reuses
  // the residual, so SURVEY's separate ~100-flop cost pass is not counted) + ~480 (local Hessian and gradient); per view
  // of camera i (i baselines in its chain) the 6-D adjoint expansion 2 (6 i + 6 + n_intr)^2 6; per frame the Schur sums
  // H_fc^T [A_f | b_f] 2 * 6 * C^2 + the 6 x 6 factorisation 6^3
  double fl = 630.0 * h->NC + F * (2.0 * 6.0 * C * C + 216.0);
  for (int v = 0; v < h->V; ++v) {
    const int i = h->vcam[v];
    const double m = 6.0 * i + 6.0 + h->d.nintr[i];
    fl += 2.0 * m * m * 6.0;
  }
  if (flops_per_launch) *flops_per_launch = fl;
  return 0;
}

int kb_build_kernel_name(kb_handle* h, char* buf, int32_t cap) {
  if (!h || !buf || cap < 1) return fail("kb_build_kernel_name: bad args");
  std::snprintf(buf, cap, "%s", h->build_pipe ? "k_buildp" : "k_build");
  return 0;
}

int kb_comm_get_unique_id(void* out) {
  if (!out) return fail("null");
  ncclUniqueId id;
  KB_NCCL(ncclGetUniqueId(&id));
  std::memcpy(out, &id, sizeof(id));
  return 0;
}

// buffers of a sharded handle (rank `rank` of `nranks`; F_max = the largest rank's frame count)
static int shard_setup(kb_handle* h, int nranks, int rank, int F_max) {
  h->nranks = nranks;
  h->rank = rank;
  h->d.rank = rank;
  // column sums widened by one max|dx_f| column per rank (GN fused passes); the one-rank buffers stay allocated
  // until kb_destroy
  h->d.Wtot = h->d.Wp + nranks;
  if (h->alloc(&h->d.part8, (size_t)kColsumRows * h->d.Wtot) || h->alloc(&h->d.psum_local, (size_t)h->d.Wtot))
    return -1;
  if (h->alloc(&h->psum_red, (size_t)h->d.Wtot)) return -1;
  double* rr = nullptr;
  if (h->alloc(&rr, 8)) return -1;
  h->d.psum = h->psum_red;
  h->d.psum_rows = 1;
  h->d.red = rr;
  double* ra = nullptr;
  if (h->alloc(&ra, 4 * (size_t)nranks)) return -1;
  h->d.red_all = ra;
  h->d.nranks = nranks;
  // per-frame step rows: padded to the largest rank's frame count (zero rows are neutral for the sums and the
  // max), all-gathered once per pass and reduced by every rank in rank order
  h->F_max = F_max;
  double* bp = nullptr;
  if (h->alloc(&bp, 4 * (size_t)h->F_max) || h->alloc(&h->bpart_all, 4 * (size_t)h->F_max * nranks)) return -1;
  h->d.bpart = bp;
  h->d.bsrc = h->bpart_all;
  h->d.bsrc_rows = h->F_max * nranks;
  if (h->alloc(&h->psum_red8, (size_t)kColsumRows * h->d.Wtot)) return -1;
  if (h->xexp && !h->ximg_part && h->alloc(&h->ximg_part, (size_t)h->d.img_n)) return -1;
  drop_graphs(h);
  KB_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

// ---------------------------------------------------------------- direct all-reduce (k_xar) setup
// KB_DIRECT_AR=0 keeps the collective (RCCL / the in-process copies) for the sharded image
static bool xar_env_on() {
  const char* e = std::getenv("KB_DIRECT_AR");
  return !(e && e[0] == '0');
}

// KB_DIRECT_AR=force (tests on a one-GPU box only): an in-process group of two members on ONE device takes the direct
// path too.  The product rule is one rank per device; two members sharing a device rely on the hardware queues
// running both members' k_xar launches at once (measured reliable for two members, not for three).
static bool xar_env_force() {
  const char* e = std::getenv("KB_DIRECT_AR");
  return e && !std::strcmp(e, "force");
}

// this rank's exchange region: flags + two image halves, zeroed (the base of its own allocation: IPC-exportable)
static int xar_region(kb_handle* h, double** out) {
  return h->alloc(out, (size_t)kXarFlagDoubles + 2 * (size_t)h->d.img_n);
}

static int xar_install(kb_handle* h, double* own, const std::vector<double*>& peers) {
  double** tab = nullptr;
  if (h->alloc(&tab, peers.size())) return -1;
  if (!h->xar_agree_buf && h->alloc(&h->xar_agree_buf, 2)) return -1;
  h->d.xar_timeout = kXarTimeoutTicks;
  if (const char* e = std::getenv("KB_XAR_TIMEOUT_MS")) {  // the wait bound of k_xar (ms; s_memrealtime runs at 100 MHz)
    const long ms = std::atol(e);
    if (ms > 0) h->d.xar_timeout = 100000ull * (unsigned long long)ms;
  }
  h->xar_failed = false;
  KB_HIP(hipMemcpyAsync(tab, peers.data(), sizeof(double*) * peers.size(), hipMemcpyHostToDevice, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  h->d.xar_buf = own;
  h->d.xar_peers = tab;
  h->d.xar = 1;
  drop_graphs(h);
  return 0;
}

static void xar_uninstall(kb_handle* h) {
  h->d.xar = 0;
  drop_graphs(h);
}

// self-test, part 1 (every rank, concurrently): known partial images, one k_xar launch
static int xar_selftest_launch(kb_handle* h) {
  unsigned long long f0 = 0;
  KB_HIP(hipMemcpyAsync(&f0, h->d.xar_buf, sizeof(f0), hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  hipLaunchKernelGGL(k_xar_fill, dim3((h->d.img_n + 255) / 256), dim3(256), 0, h->stream, h->d, (int)((f0 + 1) & 1));
  hipLaunchKernelGGL(k_xar, dim3(kXarBlocks), dim3(256), 0, h->stream, h->d, 0);
  KB_HIP(hipGetLastError());
  return 0;
}

// part 2: the exact sums arrived, no timeout; the control block's error flag cleared again
static int xar_selftest_check(kb_handle* h, int& ok) {
  std::vector<double> img(h->d.img_n);
  KbCtrl ctrl{};
  KB_HIP(hipMemcpyAsync(img.data(), h->d.simg, sizeof(double) * img.size(), hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipMemcpyAsync(&ctrl, h->d.ctrl, sizeof(KbCtrl), hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  const double R = h->nranks, base = R * (R + 1) / 2 * 0.125;
  ok = ctrl.comm_err ? 0 : 1;
  for (size_t i = 0; i < img.size() && ok; ++i) ok = img[i] == base + R * (double)(i % 7);
  const int zero = 0;
  KB_HIP(hipMemcpyAsync(&h->d.ctrl->comm_err, &zero, sizeof(int), hipMemcpyHostToDevice, h->stream));
  // both image halves back to zeros: k_colsumx writes only the image's live entries, the rest must sum to 0
  KB_HIP(hipMemsetAsync(h->d.xar_buf + kXarFlagDoubles, 0, sizeof(double) * 2 * (size_t)h->d.img_n, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

// multi-process ranks (RCCL communicator up): export this rank's region as an IPC handle, all-gather the handles and
// the ranks' PCI locations, map the peers', self-test; every step's outcome is agreed over the communicator (all ranks
// enable the direct path or none does), and every rank runs the same collectives whatever its own outcome: a local
// failure only clears `ok` (the exchange scratch is the handle's image buffer, so nothing is allocated here before the
// collectives).  The direct path needs one rank per device (distinct PCI locations); RCCL refuses two ranks on one
// device anyway, and a shared device would leave k_xar's co-scheduling to the hardware queues.
static int xar_setup_rccl(kb_handle* h) {
  if (!h->xexp || h->nranks < 2 || h->nranks > kXMaxRanksDev) return 0;
  int ok = xar_env_on() ? 1 : 0;
  double* own = nullptr;
  hipIpcMemHandle_t mh;
  std::memset(&mh, 0, sizeof(mh));
  if (ok && xar_region(h, &own)) ok = 0;
  if (ok && hipIpcGetMemHandle(&mh, own) != hipSuccess) ok = 0;
  int pci[3] = {-1, -1, -1};
  if (hipDeviceGetAttribute(&pci[0], hipDeviceAttributePciDomainID, h->device) != hipSuccess ||
      hipDeviceGetAttribute(&pci[1], hipDeviceAttributePciBusId, h->device) != hipSuccess ||
      hipDeviceGetAttribute(&pci[2], hipDeviceAttributePciDeviceId, h->device) != hipSuccess)
    ok = 0;
  hipGetLastError();
  const int loc = ((pci[0] & 0xffff) << 16) | ((pci[1] & 0xff) << 8) | (pci[2] & 0xff);
  constexpr size_t kSlot = sizeof(hipIpcMemHandle_t) + 8;
  static_assert(kSlot * (kXMaxRanksDev + 1) <= 8 * 16 * 16 * 15, "exchange scratch within the smallest C > 64 image");
  char* dx = reinterpret_cast<char*>(h->d.simg);  // scratch: the image buffer (rewritten by every pass)
  std::vector<char> slot(kSlot, 0);
  std::memcpy(slot.data(), &mh, sizeof(mh));
  std::memcpy(slot.data() + sizeof(mh), &ok, sizeof(int));
  std::memcpy(slot.data() + sizeof(mh) + sizeof(int), &loc, sizeof(int));
  if (hipMemcpyAsync(dx, slot.data(), kSlot, hipMemcpyHostToDevice, h->stream) != hipSuccess) ok = 0;
  KB_NCCL(ncclAllGather(dx, dx + kSlot, kSlot, ncclChar, h->comm, h->stream));
  std::vector<char> all(kSlot * h->nranks, 0);
  if (hipMemcpyAsync(all.data(), dx + kSlot, all.size(), hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
      hipStreamSynchronize(h->stream) != hipSuccess)
    ok = 0;
  hipGetLastError();
  std::vector<double*> peers(h->nranks, nullptr);
  std::vector<int> locs(h->nranks, 0);
  for (int q = 0; q < h->nranks && ok; ++q) {
    int okq = 0;
    std::memcpy(&okq, all.data() + kSlot * q + sizeof(mh), sizeof(int));
    std::memcpy(&locs[q], all.data() + kSlot * q + sizeof(mh) + sizeof(int), sizeof(int));
    if (!okq) ok = 0;
    for (int r = 0; r < q && ok; ++r)
      if (locs[r] == locs[q]) ok = 0;  // two ranks on one device: the collective, not the direct path
  }
  for (int q = 0; q < h->nranks && ok; ++q) {
    if (q == h->rank) {
      peers[q] = own;
      continue;
    }
    hipIpcMemHandle_t hq;
    std::memcpy(&hq, all.data() + kSlot * q, sizeof(hq));
    void* p = nullptr;
    if (hipIpcOpenMemHandle(&p, hq, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      hipGetLastError();
      ok = 0;
      break;
    }
    h->xar_opened.push_back(p);
    peers[q] = (double*)p;
  }
  auto agree = [&](int v) -> int {  // min over ranks (the collective runs whatever the copies did)
    int* di = (int*)dx;
    int r = 0;
    if (hipMemcpyAsync(di, &v, sizeof(int), hipMemcpyHostToDevice, h->stream) != hipSuccess) v = 0;
    if (ncclAllReduce(di, di, 1, ncclInt32, ncclMin, h->comm, h->stream) != ncclSuccess) return 0;
    if (hipMemcpyAsync(&r, di, sizeof(int), hipMemcpyDeviceToHost, h->stream) != hipSuccess) r = 0;
    if (hipStreamSynchronize(h->stream) != hipSuccess) r = 0;
    hipGetLastError();
    return std::min(r, v);
  };
  ok = agree(ok);
  if (ok && xar_install(h, own, peers)) ok = 0;
  ok = agree(ok);
  if (ok) {
    int t = 0;
    if (xar_selftest_launch(h) || xar_selftest_check(h, t)) t = 0;
    ok = agree(t);
  }
  if (!ok && h->d.xar) xar_uninstall(h);
  hipGetLastError();
  return 0;
}

// in-process groups: the members' regions directly (same process, peer access enabled by kb_comm_init_local).  The
// members' k_xar launches must run concurrently, which separate devices guarantee: the direct path needs one member
// per device, and a group with two members on one device keeps the copies (KB_DIRECT_AR=force lets a two-member group
// on one device take it, for the tests on a one-GPU box).  The self-test, run on every member's stream before any
// member syncs, proves the exchange before the group relies on it.
static void xar_setup_local(kb_handle* const* hs, int n) {
  if (n < 2 || n > kXMaxRanksDev || !xar_env_on()) return;
  bool distinct = true;
  for (int r = 0; r < n; ++r) {
    if (!hs[r]->xexp) return;
    for (int q = 0; q < r; ++q) distinct = distinct && hs[q]->device != hs[r]->device;
  }
  if (!distinct && !(xar_env_force() && n == 2)) return;
  std::vector<double*> regs(n, nullptr);
  for (int r = 0; r < n; ++r)
    if (hipSetDevice(hs[r]->device) != hipSuccess || xar_region(hs[r], &regs[r])) return;
  int ok = 1;
  for (int r = 0; r < n && ok; ++r)
    if (hipSetDevice(hs[r]->device) != hipSuccess || xar_install(hs[r], regs[r], regs)) ok = 0;
  for (int r = 0; r < n && ok; ++r)
    if (hipSetDevice(hs[r]->device) != hipSuccess || xar_selftest_launch(hs[r])) ok = 0;
  for (int r = 0; r < n && ok; ++r) {
    int t = 0;
    if (hipSetDevice(hs[r]->device) != hipSuccess || xar_selftest_check(hs[r], t)) t = 0;
    ok = t;
  }
  if (!ok)
    for (int r = 0; r < n; ++r) {
      hipSetDevice(hs[r]->device);
      if (hs[r]->d.xar) xar_uninstall(hs[r]);
    }
  hipGetLastError();
}

int kb_comm_direct(const kb_handle* h) { return h && h->d.xar ? 1 : 0; }

// ---- the IPC half of the direct all-reduce on its own, for a test with several processes on one GPU (RCCL refuses
// two ranks on one device, so kb_comm_init cannot be run that way): export this handle's exchange region, then map
// the peers' regions from their exported handles and run the self-test exchange (known values, rank-order sums,
// the 2 s wait bound).  The handle stays unsharded: its rank / rank count are set only for the exchange.
int kb_xar_export(kb_handle* h, void* handle_out64) {
  if (!h || !handle_out64) return fail("kb_xar_export: null");
  if (!h->xexp) return fail("kb_xar_export: the direct all-reduce needs a camera block C > 64");
  KB_HIP(hipSetDevice(h->device));
  if (!h->d.xar_buf) {
    double* own = nullptr;
    if (xar_region(h, &own)) return -1;
    KB_HIP(hipStreamSynchronize(h->stream));
    h->d.xar_buf = own;
  }
  hipIpcMemHandle_t mh;
  KB_HIP(hipIpcGetMemHandle(&mh, h->d.xar_buf));
  static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle size");
  std::memset(handle_out64, 0, 64);
  std::memcpy(handle_out64, &mh, sizeof(mh));
  return 0;
}

int kb_xar_test(kb_handle* h, int32_t nranks, int32_t rank, const void* handles64, int32_t* ok) {
  if (!h || !handles64 || !ok) return fail("kb_xar_test: null");
  if (!h->d.xar_buf) return fail("kb_xar_test: kb_xar_export first");
  if (sharded(h)) return fail("kb_xar_test: the handle is sharded");
  if (nranks < 2 || nranks > kXMaxRanksDev || rank < 0 || rank >= nranks) return fail("kb_xar_test: bad rank");
  KB_HIP(hipSetDevice(h->device));
  *ok = 0;
  std::vector<double*> peers(nranks, nullptr);
  std::vector<void*> opened;
  int rc = 0;
  for (int q = 0; q < nranks && !rc; ++q) {
    if (q == rank) {
      peers[q] = h->d.xar_buf;
      continue;
    }
    hipIpcMemHandle_t hq;
    std::memcpy(&hq, (const char*)handles64 + 64 * q, sizeof(hq));
    void* p = nullptr;
    if (hipIpcOpenMemHandle(&p, hq, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      hipGetLastError();
      rc = fail("kb_xar_test: hipIpcOpenMemHandle failed");
      break;
    }
    opened.push_back(p);
    peers[q] = (double*)p;
  }
  const KbDev saved = h->d;
  if (!rc) {
    h->d.rank = rank;
    h->d.nranks = nranks;
    h->nranks = nranks;
    h->rank = rank;
    int t = 0;
    if (xar_install(h, h->d.xar_buf, peers) || xar_selftest_launch(h) || xar_selftest_check(h, t)) rc = -1;
    *ok = t;
    h->nranks = 1;
    h->rank = 0;
  }
  const double* region = h->d.xar_buf;
  h->d = saved;
  h->d.xar_buf = const_cast<double*>(region);
  drop_graphs(h);
  for (void* p : opened) hipIpcCloseMemHandle(p);
  return rc;
}

int kb_comm_init(kb_handle* h, const void* uid, int32_t nranks, int32_t rank) {
  if (!h || !uid) return fail("kb_comm_init: null");
  KB_HIP(hipSetDevice(h->device));
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail("kb_comm_init: bad rank / nranks");
  if (sharded(h)) return fail("kb_comm_init: communicator already initialised");
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof(id));
  KB_NCCL(ncclCommInitRank(&h->comm, nranks, id, rank));
  int* fm = nullptr;
  if (h->alloc(&fm, 1)) return -1;
  KB_HIP(hipMemcpyAsync(fm, &h->F, sizeof(int), hipMemcpyHostToDevice, h->stream));
  KB_NCCL(ncclAllReduce(fm, fm, 1, ncclInt32, ncclMax, h->comm, h->stream));
  int F_max = 0;
  KB_HIP(hipMemcpyAsync(&F_max, fm, sizeof(int), hipMemcpyDeviceToHost, h->stream));
  KB_HIP(hipStreamSynchronize(h->stream));
  if (shard_setup(h, nranks, rank, F_max)) return -1;
  return xar_setup_rccl(h);
}

int kb_comm_init_local(kb_handle* const* hs, int32_t n) {
  if (!hs || n < 1 || n > kLocalMaxRanks) return fail("kb_comm_init_local: bad handle list");
  int F_max = 0;
  for (int r = 0; r < n; ++r) {
    if (!hs[r]) return fail("kb_comm_init_local: null handle");
    if (sharded(hs[r])) return fail("kb_comm_init_local: handle already sharded");
    for (int q = 0; q < r; ++q)
      if (hs[q] == hs[r]) return fail("kb_comm_init_local: handle listed twice");
    if (hs[r]->N != hs[0]->N || hs[r]->C != hs[0]->C) return fail("kb_comm_init_local: handles of different rigs");
    F_max = std::max(F_max, hs[r]->F);
  }
  // the group's kernels read every member's send buffer from their own device: members on different devices need
  // peer access both ways (enabled here; groups whose devices cannot reach each other are refused)
  for (int r = 0; r < n; ++r)
    for (int q = 0; q < n; ++q) {
      const int a = hs[r]->device, b = hs[q]->device;
      if (a == b) continue;
      int can = 0;
      KB_HIP(hipDeviceCanAccessPeer(&can, a, b));
      if (!can) return fail("kb_comm_init_local: devices of the group cannot access each other's memory");
      KB_HIP(hipSetDevice(a));
      const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
        return fail(std::string("kb_comm_init_local: hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
      hipGetLastError();
    }
  // everything that can fail runs before any handle joins: on failure the handles stay unsharded and usable
  kb_local_group* G = new kb_local_group();
  G->n = n;
  G->ready.assign(n, nullptr);
  G->done.assign(n, nullptr);
  G->src.assign(n, nullptr);
  auto drop_group = [&]() {
    for (auto e : G->ready)
      if (e) hipEventDestroy(e);
    for (auto e : G->done)
      if (e) hipEventDestroy(e);
    delete G;
  };
  for (int r = 0; r < n; ++r) {
    if (hipSetDevice(hs[r]->device) != hipSuccess ||
        hipEventCreateWithFlags(&G->ready[r], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&G->done[r], hipEventDisableTiming) != hipSuccess) {
      drop_group();
      return fail("kb_comm_init_local: event creation failed");
    }
  }
  struct Saved {
    KbDev d;
    int nranks, rank, F_max;
    double *psum_red, *psum_red8, *bpart_all;
  };
  std::vector<Saved> saved(n);
  for (int r = 0; r < n; ++r) {
    kb_handle* h = hs[r];
    saved[r] = Saved{h->d, h->nranks, h->rank, h->F_max, h->psum_red, h->psum_red8, h->bpart_all};
  }
  for (int r = 0; r < n; ++r) {
    if (hipSetDevice(hs[r]->device) != hipSuccess || shard_setup(hs[r], n, r, F_max)) {
      for (int q = 0; q <= r; ++q) {  // roll back (buffers already allocated stay with the handle until kb_destroy)
        kb_handle* h = hs[q];
        const Saved& sv = saved[q];
        h->d = sv.d;
        h->nranks = sv.nranks;
        h->rank = sv.rank;
        h->F_max = sv.F_max;
        h->psum_red = sv.psum_red;
        h->psum_red8 = sv.psum_red8;
        h->bpart_all = sv.bpart_all;
        drop_graphs(h);
      }
      drop_group();
      return fail(std::string("kb_comm_init_local: shard setup failed: ") + kb_last_error());
    }
  }
  for (int r = 0; r < n; ++r) {  // publish: from here on the handles are ranks of the group
    hs[r]->lg = G;
    ++G->refs;
  }
  xar_setup_local(hs, n);
  return 0;
}

#ifdef KB_STAMPS
// diagnostic build only: the KB_TS timeline of the last k_solve launch (100 MHz ticks)
int kb_diag_read_ts(kb_handle* h, long long* out, int n) {
  if (!h->d.dbg_ts) {
    KB_HIP(hipMalloc(&h->d.dbg_ts, 256 * sizeof(long long)));
    KB_HIP(hipMemset(h->d.dbg_ts, 0, 256 * sizeof(long long)));
    drop_graphs(h);
    return 0;
  }
  KB_HIP(hipMemcpy(out, h->d.dbg_ts, sizeof(long long) * std::min(n, 256), hipMemcpyDeviceToHost));
  return 0;
}

// diagnostic build only: the dbg_flags every later launch of the handle's kernels sees (k_marg: bit 1 skips the
// rounds' work, bit 2 skips the rotations)
int kb_diag_set_flags(kb_handle* h, int flags) {
  h->d.dbg_flags = flags;
  drop_graphs(h);
  return 0;
}

// diagnostic build only: average duration (us, HIP events over `reps` launches) of one kernel of the GN pass run
// up to stop point `stop` (KB_STAMP): which = 0 fused build, 1 camera solve, 2 back-substitution, 3 GN fused build.
int kb_diag_phase_time(kb_handle* h, int which, int stop, int reps, int flags, double* us) {
  KB_HIP(hipSetDevice(h->device));
  KbOpts o{1, 0x3fffffff, 0.0, -1.0, -1.0};
  if (ensure_trace(h, 64) || loop_start(h, o)) return -1;
  for (int i = 0; i < 2; ++i)
    if (enqueue_pass(h, 1)) return -1;
  if (launch_build(h, 0, 1) || launch_colsum(h, 0, false)) return -1;
  KbDev d = h->d;
  d.dbg_stop = stop;
  d.dbg_flags = flags;
  d.psum = d.part8;
  d.psum_rows = kColsumRows;
  hipEvent_t e0, e1;
  KB_HIP(hipEventCreate(&e0));
  KB_HIP(hipEventCreate(&e1));
  int g = 0, one = 1, zero = 0;
  for (int r = -2; r < reps; ++r) {
    if (r == 0) KB_HIP(hipEventRecord(e0, h->stream));
    if (which == 0) {
      void* args[] = {&d, &g, &one};
      KB_HIP(hipLaunchKernel(h->fn_build, dim3(d.nblk), dim3(h->build_threads), args, h->lds_build, h->stream));
    } else if (which == 3) {  // GN fused build (gated: applies the pending frame steps each launch)
      KbDev dg = d;
      dg.gn_fused = 1;
      dg.fold = 0;
      void* args[] = {&dg, &one, &one};
      KB_HIP(hipLaunchKernel(h->fn_build_gn, dim3(d.nblk), dim3(h->build_threads), args, h->lds_build, h->stream));
    } else if (which == 1) {
      void* args[] = {&d, &g, &zero};
      KB_HIP(hipLaunchKernel(h->fn_solve, dim3(1), dim3(h->solve_threads), args, h->lds_solve, h->stream));
    } else {
      hipLaunchKernelGGL(k_backsub, dim3((h->F + kBsFrames - 1) / kBsFrames), dim3(64 * kBsFrames), 0, h->stream, d, 0, 1,
                         1);
    }
  }
  KB_HIP(hipEventRecord(e1, h->stream));
  KB_HIP(hipEventSynchronize(e1));
  float ms = 0.f;
  KB_HIP(hipEventElapsedTime(&ms, e0, e1));
  *us = 1e3 * ms / reps;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return 0;
}
#endif

int kb_selftest_mfma(double* max_err) {
  double* d = nullptr;
  KB_HIP(hipMalloc(&d, sizeof(double) * 256));
  double worst = 0.0;
  for (int ident = 1; ident >= 0; --ident) {
    hipLaunchKernelGGL(k_selftest_mfma, dim3(1), dim3(64), 0, 0, d, ident);
    KB_HIP(hipGetLastError());
    double hD[256];
    KB_HIP(hipMemcpy(hD, d, sizeof(hD), hipMemcpyDeviceToHost));
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double s = 0.0;
        for (int k = 0; k < 16; ++k) {
          const double a = ident ? (i == k ? 1.0 : 0.0) : (i * 0.5 + k * 0.125 + ((i * 3 + k) % 5));
          const double b = k * 16.0 + j + 0.25 * ((k * 5 + j * 3) % 7);
          s += a * b;
        }
        worst = std::max(worst, std::fabs(s - hD[i * 16 + j]));
      }
  }
  hipFree(d);
  if (max_err) *max_err = worst;
  return 0;
}

}  // extern "C"
