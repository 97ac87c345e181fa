// Stream-capture state probe (diagnostic for the r03 libamdhip64 stack overflow).
//
// The render library records the same fork/join events (ev_fork, ev_join, ...) inside stream captures
// (on its capture streams) and in direct launches (on its direct streams).  This probe replays that
// pattern and prints, after every step, which streams the runtime believes are capturing:
//   step a: capture on `cap`: record ev_fork, cap_side waits it, kernel on cap_side, record ev_join on
//           cap_side, cap waits it; end capture, instantiate, launch on `main`;
//   step b: direct: record ev_fork on `main`, `side` waits it, kernel, record ev_join on side, main waits.
// Mode 0 shares the two events between a and b (the r03 library); mode 1 gives each its own pair.
// Built as a shared object (extern "C" probe_run) so that it can run against the libamdhip64 torch
// loads (the library the crash was seen in) or the ROCm one.
#include <hip/hip_runtime.h>
#include <execinfo.h>
#include <csignal>
#include <cstdio>

// a host SIGSEGV prints the native backtrace (to compare with the library's r03 crash frames)
static void segv_bt(int sig) {
  void* fr[24];
  const int n = backtrace(fr, 24);
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
__attribute__((constructor)) static void install_segv_bt() {
  void* prime[2];
  (void)backtrace(prime, 2);
  static char alt[1 << 16];
  stack_t ss{};
  ss.ss_sp = alt;
  ss.ss_size = sizeof(alt);
  sigaltstack(&ss, nullptr);
  struct sigaction sa{};
  sa.sa_handler = segv_bt;
  sa.sa_flags = SA_ONSTACK;
  sigaction(SIGSEGV, &sa, nullptr);
}

__global__ void k_touch(int* p, int v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += v;
}

static const char* cap_name(hipStreamCaptureStatus s) {
  return s == hipStreamCaptureStatusNone ? "none" : s == hipStreamCaptureStatusActive ? "ACTIVE" : "INVALIDATED";
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("  %s -> %s\n", #x, hipGetErrorString(e_));                  \
      return 1;                                                                \
    }                                                                          \
  } while (0)

extern "C" int probe_run(int mode, int iters, int verbose) {
  hipStream_t cap, cap_side, main_s, side;
  CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&cap_side, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&main_s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
  hipEvent_t ef[2], ej[2];
  for (int i = 0; i < 2; ++i) {
    CK(hipEventCreateWithFlags(&ef[i], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ej[i], hipEventDisableTiming));
  }
  int* d = nullptr;
  CK(hipMalloc(&d, 64));
  CK(hipMemset(d, 0, 64));
  hipStream_t all[4] = {cap, cap_side, main_s, side};
  const char* names[4] = {"cap", "cap_side", "main", "side"};
  int stale = 0;
  auto report = [&](const char* step, int it) {
    int bad = 0;
    for (int i = 0; i < 4; ++i) {
      hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
      (void)hipStreamIsCapturing(all[i], &st);
      if (st != hipStreamCaptureStatusNone) ++bad;
      if (verbose || st != hipStreamCaptureStatusNone) std::printf("  iter %d after %s: %s %s\n", it, step, names[i], cap_name(st));
    }
    return bad;
  };
  for (int it = 0; it < iters; ++it) {
    // a: capture
    hipEvent_t f = ef[0], j = ej[0];
    CK(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
    k_touch<<<1, 64, 0, cap>>>(d, 1);
    CK(hipEventRecord(f, cap));
    CK(hipStreamWaitEvent(cap_side, f, 0));
    k_touch<<<1, 64, 0, cap_side>>>(d + 1, 1);
    CK(hipEventRecord(j, cap_side));
    CK(hipStreamWaitEvent(cap, j, 0));
    hipGraph_t g = nullptr;
    CK(hipStreamEndCapture(cap, &g));
    hipGraphExec_t ge = nullptr;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, main_s));
    stale += report("capture", it);
    // b: direct launches on other streams
    if (mode == 1) f = ef[1], j = ej[1];
    CK(hipEventRecord(f, main_s));
    CK(hipStreamWaitEvent(side, f, 0));
    k_touch<<<1, 64, 0, side>>>(d + 2, 1);
    CK(hipEventRecord(j, side));
    CK(hipStreamWaitEvent(main_s, j, 0));
    stale += report("direct", it);
    CK(hipStreamSynchronize(main_s));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  int h[3] = {0, 0, 0};
  CK(hipMemcpy(h, d, 12, hipMemcpyDeviceToHost));
  std::printf("mode %d: %d iterations, counters %d %d %d, stale capturing-stream reports %d\n", mode, iters, h[0], h[1], h[2],
              stale);
  for (hipStream_t s : all) (void)hipStreamDestroy(s);
  for (int i = 0; i < 2; ++i) {
    (void)hipEventDestroy(ef[i]);
    (void)hipEventDestroy(ej[i]);
  }
  (void)hipFree(d);
  return stale;
}

// Topologies of one capture on origin O with three more streams A, B, L (probe_topo):
//   1  A and B fork from O; B waits an event of A, then A waits an event of B (side <-> side); join
//   2  L forks from O, A forks from L (nested fork), A joins L, L joins O
//   3  L forks from O, A forks from O; A waits an event of L, L waits an event of A (lane <-> side)
//   4  the r03 two-lane call: lane 0 on O with side A, lane 1 on L with side B, three sample batches,
//      each k_sky after the previous batch's (cross waits A <-> B), k_accum after the previous (O <-> L)
// After the capture ends, every stream's capture status is printed; a stale ACTIVE status (or a crash)
// names the topology the runtime mishandles.
extern "C" int probe_topo(int topo, int iters) {
  hipStream_t O, A, B, L;
  CK(hipStreamCreateWithFlags(&O, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&L, hipStreamNonBlocking));
  hipEvent_t e[8];
  for (auto& x : e) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  int* d = nullptr;
  CK(hipMalloc(&d, 256));
  CK(hipMemset(d, 0, 256));
  hipStream_t all[4] = {O, A, B, L};
  const char* names[4] = {"O", "A", "B", "L"};
  auto fork = [&](hipStream_t from, hipStream_t to, hipEvent_t ev) {
    hipError_t r = hipEventRecord(ev, from);
    if (r == hipSuccess) r = hipStreamWaitEvent(to, ev, 0);
    return r;
  };
  int stale = 0;
  for (int it = 0; it < iters; ++it) {
    CK(hipStreamBeginCapture(O, hipStreamCaptureModeThreadLocal));
    k_touch<<<1, 64, 0, O>>>(d, 1);
    if (topo == 1) {
      CK(fork(O, A, e[0]));
      CK(fork(O, B, e[1]));
      k_touch<<<1, 64, 0, A>>>(d + 1, 1);
      CK(fork(A, B, e[2]));
      k_touch<<<1, 64, 0, B>>>(d + 2, 1);
      CK(fork(B, A, e[3]));
      k_touch<<<1, 64, 0, A>>>(d + 1, 1);
      CK(fork(A, O, e[4]));
      CK(fork(B, O, e[5]));
    } else if (topo == 2) {
      CK(fork(O, L, e[0]));
      CK(fork(L, A, e[1]));
      k_touch<<<1, 64, 0, A>>>(d + 1, 1);
      CK(fork(A, L, e[2]));
      k_touch<<<1, 64, 0, L>>>(d + 3, 1);
      CK(fork(L, O, e[3]));
    } else if (topo == 3) {
      CK(fork(O, L, e[0]));
      CK(fork(O, A, e[1]));
      k_touch<<<1, 64, 0, L>>>(d + 3, 1);
      CK(fork(L, A, e[2]));
      k_touch<<<1, 64, 0, A>>>(d + 1, 1);
      CK(fork(A, L, e[3]));
      k_touch<<<1, 64, 0, L>>>(d + 3, 1);
      CK(fork(L, O, e[4]));
    } else if (topo == 4) {
      hipStream_t main_s[2] = {O, L}, side[2] = {A, B};
      hipEvent_t ev_fork[2] = {e[0], e[1]}, ev_sky[2] = {e[2], e[3]}, ev_acc[2] = {e[4], e[5]};
      bool sky_rec[2] = {false, false}, acc_rec[2] = {false, false};
      CK(fork(O, L, e[6]));  // ev_lane
      for (int b = 0; b < 3; ++b) {
        const int j = b & 1;
        hipStream_t ms = main_s[j], ss = side[j];
        CK(hipEventRecord(ev_fork[j], ms));
        k_touch<<<1, 64, 0, ms>>>(d + 4 + j, 1);  // trace
        CK(hipStreamWaitEvent(ss, ev_fork[j], 0));
        if (sky_rec[1 - j]) CK(hipStreamWaitEvent(ss, ev_sky[1 - j], 0));
        k_touch<<<1, 64, 0, ss>>>(d + 6, 1);  // k_sky
        CK(hipEventRecord(ev_sky[j], ss));
        sky_rec[j] = true;
        CK(hipStreamWaitEvent(ms, ev_sky[j], 0));
        if (acc_rec[1 - j]) CK(hipStreamWaitEvent(ms, ev_acc[1 - j], 0));
        k_touch<<<1, 64, 0, ms>>>(d + 7, 1);  // k_accum
        CK(hipEventRecord(ev_acc[j], ms));
        acc_rec[j] = true;
      }
      CK(hipStreamWaitEvent(O, ev_acc[1], 0));
    }
    std::printf("topo %d iter %d: ending capture\n", topo, it);
    std::fflush(stdout);
    hipGraph_t g = nullptr;
    const hipError_t ec = hipStreamEndCapture(O, &g);
    std::printf("topo %d iter %d: end capture -> %s\n", topo, it, hipGetErrorString(ec));
    for (int i = 0; i < 4; ++i) {
      hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
      (void)hipStreamIsCapturing(all[i], &st);
      if (st != hipStreamCaptureStatusNone) {
        ++stale;
        std::printf("  stream %s still %s\n", names[i], cap_name(st));
      }
    }
    std::fflush(stdout);
    if (ec == hipSuccess && g) {
      size_t n = 0, ne = 0;
      (void)hipGraphGetNodes(g, nullptr, &n);
      (void)hipGraphGetEdges(g, nullptr, nullptr, &ne);
      hipGraphExec_t ge = nullptr;
      const hipError_t ei = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
      std::printf("  graph: %zu nodes, %zu edges, instantiate %s\n", n, ne, hipGetErrorString(ei));
      if (ei == hipSuccess) {
        CK(hipGraphLaunch(ge, O));
        CK(hipStreamSynchronize(O));
        CK(hipGraphExecDestroy(ge));
      }
      CK(hipGraphDestroy(g));
    }
  }
  std::printf("topo %d: stale %d\n", topo, stale);
  for (hipStream_t s : all) (void)hipStreamDestroy(s);
  for (auto& x : e) (void)hipEventDestroy(x);
  (void)hipFree(d);
  return stale;
}
