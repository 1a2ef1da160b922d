// The chip's VALU issue rate for wave64 v_fma_f32 / v_pk_fma_f32 at 1, 2, 4 and 8 waves per SIMD
// (is the FP32 VALU peak of SQ_INSTS_VALU x 64 the 78.6 T lane-instr/s of a 2-cycle
// wave64 issue, or the 39.3 T that one wave alone reaches at ~4.9 cycles?). Each wave runs 8
// independent chains of 64 x 128 asm instructions; the grid is 256 x W workgroups of 256 threads
// (W waves per SIMD when every CU holds W workgroups: the kernel uses ~40 VGPRs). Reported per W:
// s_memtime cycles per instruction seen by one wave, and the whole chip's wave-instructions per
// second from HIP events around the launch (x 64 = lane-instructions / s).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_occupancy_probe tools/valu_occupancy_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
#define REP16(X) X X X X X X X X X X X X X X X X

template <int K>
__global__ void __launch_bounds__(256) probe(float* out, long long* cyc, int iters) {
  f2 a[8], b = {1.0001f, 0.9999f}, c = {1e-7f, 2e-7f};
  float s[8], sb = 1.0001f, sc = 1e-7f;
  for (int i = 0; i < 8; i++) {
    a[i] = f2{(float)threadIdx.x + i, (float)i};
    s[i] = (float)threadIdx.x + i;
  }
  __syncthreads();
  const long long t0 = clock64();
  for (int it = 0; it < iters; it++) {
    if constexpr (K == 0) {
#define I0(j) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s[j]) : "v"(sb), "v"(sc));
      REP16(I0(0) I0(1) I0(2) I0(3) I0(4) I0(5) I0(6) I0(7))
    } else {
#define I1(j) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
      REP16(I1(0) I1(1) I1(2) I1(3) I1(4) I1(5) I1(6) I1(7))
    }
  }
  const long long t1 = clock64();
  float acc = 0.0f;
  for (int i = 0; i < 8; i++) acc += s[i] + a[i].x + a[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int K>
static void run(const char* name, int ncu, int W, float* out, long long* cyc_d, int iters) {
  const int nb = ncu * W;
  std::vector<long long> h((size_t)nb * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(probe<K>, dim3(nb), dim3(256), 0, 0, out, cyc_d, iters);  // warm the clock
  hipLaunchKernelGGL(probe<K>, dim3(nb), dim3(256), 0, 0, out, cyc_d, iters);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(probe<K>, dim3(nb), dim3(256), 0, 0, out, cyc_d, iters);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipMemcpy(h.data(), cyc_d, sizeof(long long) * h.size(), hipMemcpyDeviceToHost);
  double s = 0;
  for (long long v : h) s += (double)v;
  const double per_wave = s / h.size() / (iters * 128.0);
  const double winst = (double)nb * 4 * iters * 128.0;
  printf("  %-14s W=%d  %6.2f cyc/instr per wave  %7.2f T lane-instr/s chip (%.3f ms)\n", name, W, per_wave,
         winst * 64 / (ms * 1e-3) / 1e12, ms);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int ncu = p.multiProcessorCount, iters = 4000;
  printf("%d CUs, wave64 VALU issue vs waves per SIMD (W workgroups of 4 waves per CU)\n", ncu);
  float* out;
  long long* cyc_d;
  hipMalloc(&out, sizeof(float) * ncu * 8 * 256);
  hipMalloc(&cyc_d, sizeof(long long) * ncu * 8 * 4);
  for (int W : {1, 2, 4, 8}) run<0>("v_fma_f32", ncu, W, out, cyc_d, iters);
  for (int W : {1, 2, 4}) run<1>("v_pk_fma_f32", ncu, W, out, cyc_d, iters);
  printf("status: %s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
