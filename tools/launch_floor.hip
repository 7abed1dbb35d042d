// launch_floor.hip -- development microbenchmark (not shipped, not a test):
// what one dependent kernel boundary costs on MI355X in the update's own
// capture mode, measured two ways: event time per kernel of a chain, and the
// in-kernel span clock (s_memrealtime, 100 MHz, one counter for the chip):
// each wave stores (first instruction, exit) -- so a boundary's idle time is
// the next kernel's first wave start minus the previous kernel's last wave
// exit, and a kernel's span is its last exit minus its first start.
//
// Varied:
//   (i)   the launch form: eager back-to-back launches (queued behind a spin),
//         and a hipGraph captured from the stream (what torch.cuda.graph and the
//         C host both build: stream capture -> hipGraphInstantiate -> launch);
//   (ii)  the predecessor's dirty bytes: a kernel that writes 0 / 2.8 MB (Adam's
//         P, M, V, W2T) / 25 MB (the rowpass's k-packed planes) before a trivial
//         kernel;
//   (iii) nodes per graph: 4 / 16 / 64 / 256.
// Every kernel runs 256 workgroups of 256 threads (one per CU, like the
// update's reduce / Adam / dW2 launches).
// Output: one JSON object on stdout.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/launch_floor.hip -o tools/_probe/launch_floor
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

constexpr int kBlocks = 256, kThreads = 256, kWaves = kBlocks * kThreads / 64;

__device__ __forceinline__ void stamp(unsigned long long* rec, unsigned long long t0) {
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) {
    const int wv = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    *reinterpret_cast<ulonglong2*>(rec + 2 * wv) = make_ulonglong2(t0, t1);
  }
}

// writes n4 float4 (grid-stride): leaves that many bytes dirty in L2 for the
// next kernel's boundary
__global__ void __launch_bounds__(kThreads) dirty_kernel(float4* buf, long long n4, float v, unsigned long long* rec) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x)
    buf[i] = make_float4(v, v, v, v);
  stamp(rec, t0);
}

__global__ void __launch_bounds__(kThreads) noop_kernel(unsigned long long* rec) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  stamp(rec, t0);
}

__global__ void spin_kernel(long long cycles) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
}

struct Launch {
  bool dirty;
  unsigned long long* rec;
};

// one chain: n launches; with dirty_bytes > 0 every other launch is the dirty kernel
static void enqueue(hipStream_t s, const std::vector<Launch>& ch, float4* buf, long long n4) {
  for (const Launch& l : ch) {
    if (l.dirty)
      hipLaunchKernelGGL(dirty_kernel, dim3(kBlocks), dim3(kThreads), 0, s, buf, n4, 1.0f, l.rec);
    else
      hipLaunchKernelGGL(noop_kernel, dim3(kBlocks), dim3(kThreads), 0, s, l.rec);
  }
}

struct Result {
  double event_us_per_kernel, span_noop_us, span_dirty_us, gap_after_dirty_us, gap_after_noop_us;
};

static Result analyse(const std::vector<Launch>& ch, unsigned long long* host, unsigned long long* dev, size_t words,
                      double event_us) {
  CK(hipMemcpy(host, dev, words * 8, hipMemcpyDeviceToHost));
  std::vector<std::pair<unsigned long long, unsigned long long>> se;
  for (const Launch& l : ch) {
    const unsigned long long* r = host + (l.rec - dev);
    unsigned long long a = ~0ull, b = 0;
    for (int w = 0; w < kWaves; ++w) {
      a = std::min(a, r[2 * w]);
      b = std::max(b, r[2 * w + 1]);
    }
    se.emplace_back(a, b);
  }
  double sn = 0, sd = 0, gd = 0, gn = 0;
  int nn = 0, nd = 0, ngd = 0, ngn = 0;
  for (size_t i = 0; i < ch.size(); ++i) {
    const double span = (se[i].second - se[i].first) * 0.01;
    if (ch[i].dirty) { sd += span; ++nd; } else { sn += span; ++nn; }
    if (i + 1 < ch.size()) {
      const double gap = ((long long)se[i + 1].first - (long long)se[i].second) * 0.01;
      if (ch[i].dirty) { gd += gap; ++ngd; } else { gn += gap; ++ngn; }
    }
  }
  return Result{event_us, nn ? sn / nn : 0, nd ? sd / nd : 0, ngd ? gd / ngd : 0, ngn ? gn / ngn : 0};
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const long long max_bytes = 25LL << 20;
  float4* buf;
  CK(hipMalloc(&buf, max_bytes));
  const int max_nodes = 256;
  const size_t words = (size_t)max_nodes * kWaves * 2;
  unsigned long long *rec, *host;
  CK(hipMalloc(&rec, words * 8));
  host = (unsigned long long*)std::malloc(words * 8);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("{\"tool\": \"tools/launch_floor.hip\", \"blocks\": %d, \"threads\": %d, \"rows\": [\n", kBlocks, kThreads);
  bool first = true;
  const long long dirty_sizes[3] = {0, 2900000LL, 25165824LL};   // 0, Adam's ~2.8 MB, the rowpass's 25.2 MB planes
  const int node_counts[4] = {4, 16, 64, 256};
  for (int form = 0; form < 2; ++form) {
    for (long long db : dirty_sizes) {
      for (int nodes : node_counts) {
        if (form == 0 && nodes != 64) continue;            // eager: one chain length
        std::vector<Launch> ch;
        for (int k = 0; k < nodes; ++k) ch.push_back(Launch{db > 0 && (k % 2 == 0), rec + (size_t)k * kWaves * 2});
        const long long n4 = db / 16;
        float ev_us = 0;
        if (form == 0) {
          enqueue(s, ch, buf, n4);                         // warm-up
          CK(hipStreamSynchronize(s));
          hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(1), 0, s, 20000000LL);   // host runs ahead
          CK(hipEventRecord(e0, s));
          enqueue(s, ch, buf, n4);
          CK(hipEventRecord(e1, s));
        } else {
          hipGraph_t g;
          hipGraphExec_t ge;
          CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
          enqueue(s, ch, buf, n4);
          CK(hipStreamEndCapture(s, &g));
          CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
          for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
          CK(hipStreamSynchronize(s));
          CK(hipEventRecord(e0, s));
          CK(hipGraphLaunch(ge, s));
          CK(hipEventRecord(e1, s));
          CK(hipStreamSynchronize(s));
          CK(hipGraphExecDestroy(ge));
          CK(hipGraphDestroy(g));
        }
        CK(hipStreamSynchronize(s));
        CK(hipEventElapsedTime(&ev_us, e0, e1));
        const Result r = analyse(ch, host, rec, words, ev_us * 1e3 / nodes);
        std::printf("%s  {\"form\": \"%s\", \"predecessor_dirty_bytes\": %lld, \"nodes\": %d, "
                    "\"event_us_per_kernel\": %.3f, \"span_trivial_us\": %.3f, \"span_dirty_us\": %.3f, "
                    "\"gap_after_trivial_us\": %.3f, \"gap_after_dirty_us\": %.3f}",
                    first ? "" : ",\n", form == 0 ? "eager" : "stream_capture_graph", db, nodes, r.event_us_per_kernel,
                    r.span_noop_us, r.span_dirty_us, r.gap_after_noop_us, r.gap_after_dirty_us);
        first = false;
      }
    }
  }
  std::printf("\n]}\n");
  return 0;
}
