// Launch cost probe: a chain of small dependent kernels launched directly on
// a stream, against the same chain captured once into a hipGraph and replayed.
// Prints the wall time per kernel of each (after warm-up).
// build: hipcc --offload-arch=gfx950 -O2 tools/graph_probe.hip -o tools/_graph_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                 \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

// one workgroup-sized chunk of work per block: a few loads and stores
__global__ void __launch_bounds__(256) k_step(double* a, int n, double s) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = a[i] * s + 1.0;
}

int main(int argc, char** argv) {
  const int chain = argc > 1 ? std::atoi(argv[1]) : 60;
  const int blocks = argc > 2 ? std::atoi(argv[2]) : 8;
  const int reps = 50;
  const int n = blocks * 256;
  double* a;
  CHK(hipMalloc(&a, sizeof(double) * n));
  CHK(hipMemset(a, 0, sizeof(double) * n));
  hipStream_t st;
  CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  auto run_chain = [&] {
    for (int k = 0; k < chain; k++) k_step<<<blocks, 256, 0, st>>>(a, n, 0.5);
  };
  for (int w = 0; w < 5; w++) run_chain();
  CHK(hipStreamSynchronize(st));
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; r++) run_chain();
  CHK(hipStreamSynchronize(st));
  auto t1 = std::chrono::steady_clock::now();
  const double direct = std::chrono::duration<double, std::micro>(t1 - t0).count() / (reps * chain);

  hipGraph_t g;
  hipGraphExec_t ge;
  CHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  run_chain();
  CHK(hipStreamEndCapture(st, &g));
  CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int w = 0; w < 5; w++) CHK(hipGraphLaunch(ge, st));
  CHK(hipStreamSynchronize(st));
  t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; r++) CHK(hipGraphLaunch(ge, st));
  CHK(hipStreamSynchronize(st));
  t1 = std::chrono::steady_clock::now();
  const double graph = std::chrono::duration<double, std::micro>(t1 - t0).count() / (reps * chain);

  // capture + exec update + launch every time (arguments may change per call)
  t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; r++) {
    hipGraph_t g2;
    CHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    run_chain();
    CHK(hipStreamEndCapture(st, &g2));
    hipGraphExecUpdateResult res;
    hipGraphNode_t err_node;
    CHK(hipGraphExecUpdate(ge, g2, &err_node, &res));
    CHK(hipGraphLaunch(ge, st));
    CHK(hipGraphDestroy(g2));
  }
  CHK(hipStreamSynchronize(st));
  t1 = std::chrono::steady_clock::now();
  const double upd = std::chrono::duration<double, std::micro>(t1 - t0).count() / (reps * chain);

  // host cost of issuing the direct chain (no wait)
  t0 = std::chrono::steady_clock::now();
  run_chain();
  t1 = std::chrono::steady_clock::now();
  const double issue = std::chrono::duration<double, std::micro>(t1 - t0).count() / chain;
  CHK(hipStreamSynchronize(st));
  std::printf("chain %d blocks %d: us per kernel  direct %.2f  graph %.2f  capture+update+graph %.2f  "
              "(host issue %.2f)\n", chain, blocks, direct, graph, upd, issue);
  return 0;
}
