// Probe: the wall time of a C4-like round of four dependent kernels (busy-wait kernels of
// 6, 38, 12 and 15 us) with a host synchronisation per round, launched one by one against
// replayed as a captured hipGraph (with and without a kernel-node parameter update per
// round).  Tells whether a graph shortens the round's exposed host time on this ROCm.
// build: hipcc --offload-arch=gfx950 -O2 tools/graph_launch_probe.hip -o tools/graph_launch_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

struct Args {
  unsigned long long ticks;  // wall-clock ticks (100 MHz) to spin
  unsigned* sink;
  unsigned round;
};

__global__ void k_spin(Args a) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < a.ticks) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0 && blockIdx.x == 0) a.sink[0] = a.round;
}

int main(int argc, char** argv) {
  // argv[1]: kernels per round (1-4; the same 71 us of busy time split over them)
  const int nk = argc > 1 ? std::max(1, std::min(4, atoi(argv[1]))) : 4;
  unsigned* sink;
  CK(hipMalloc(&sink, 64));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  unsigned long long us[4] = {6, 38, 12, 15};
  if (nk == 3) { us[0] = 44; us[1] = 12; us[2] = 15; }
  if (nk == 2) { us[0] = 44; us[1] = 27; }
  if (nk == 1) us[0] = 71;
  const int blocks[4] = {1024, 1563, 256, 512};
  const int R = 2000;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto launch_all = [&](unsigned r) -> hipError_t {
    for (int k = 0; k < nk; k++) {
      hipLaunchKernelGGL(k_spin, dim3(blocks[k]), dim3(256), 0, st, Args{us[k] * 100, sink, r});
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  };
  for (int w = 0; w < 50; w++) {
    CK(launch_all(w));
    CK(hipStreamSynchronize(st));
  }
  // 1. launches
  std::vector<double> t1;
  for (int r = 0; r < R; r++) {
    const auto a = now();
    CK(launch_all(r));
    CK(hipStreamSynchronize(st));
    t1.push_back(std::chrono::duration<double, std::micro>(now() - a).count());
  }
  // 2. graph replay
  hipGraph_t g;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  CK(launch_all(0));
  CK(hipStreamEndCapture(st, &g));
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  size_t nn = 0;
  CK(hipGraphGetNodes(g, nullptr, &nn));
  std::vector<hipGraphNode_t> nodes(nn);
  CK(hipGraphGetNodes(g, nodes.data(), &nn));
  for (int w = 0; w < 50; w++) {
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
  }
  std::vector<double> t2, t3;
  for (int r = 0; r < R; r++) {
    const auto a = now();
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    t2.push_back(std::chrono::duration<double, std::micro>(now() - a).count());
  }
  // 3. graph replay with one kernel-node parameter update per node per round
  for (int r = 0; r < R; r++) {
    const auto a = now();
    for (size_t k = 0; k < nn; k++) {
      hipKernelNodeParams p{};
      CK(hipGraphKernelNodeGetParams(nodes[k], &p));
      Args na{us[k % nk] * 100, sink, (unsigned)r};
      void* args[] = {&na};
      p.kernelParams = args;
      CK(hipGraphExecKernelNodeSetParams(ge, nodes[k], &p));
    }
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    t3.push_back(std::chrono::duration<double, std::micro>(now() - a).count());
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  printf("{\"kernels\": %d, \"busy_us\": %d, \"launches_us\": %.2f, \"graph_us\": %.2f, \"graph_setparams_us\": %.2f}\n",
         nk, (int)(us[0] + us[1] + us[2] + us[3]) * 0 + 71, med(t1), med(t2), med(t3));
  return 0;
}
