// One wave per SIMD (256 threads, one workgroup per CU): the issue cost of a stream of independent
// VALU instructions for one wave alone, in shader cycles per instruction (s_memtime around a
// 64 x 16-instruction loop). Measures v_fma_f32 against the packed fp32 forms and the
// transcendentals, to decide whether packed math doubles a one-wave-per-SIMD kernel's FMA rate.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_issue_probe tools/valu_issue_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

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
    if constexpr (K == 0) {  // v_fma_f32, 8 independent chains
#define I0(j) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s[j]) : "v"(sb), "v"(sc));
      REP16(I0(0) I0(1) I0(2) I0(3) I0(4) I0(5) I0(6) I0(7))
    } else if constexpr (K == 1) {  // v_pk_fma_f32, 8 independent chains
#define I1(j) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
      REP16(I1(0) I1(1) I1(2) I1(3) I1(4) I1(5) I1(6) I1(7))
    } else if constexpr (K == 2) {  // v_pk_mul_f32
#define I2(j) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      REP16(I2(0) I2(1) I2(2) I2(3) I2(4) I2(5) I2(6) I2(7))
    } else if constexpr (K == 3) {  // v_pk_add_f32
#define I3(j) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[j]) : "v"(c));
      REP16(I3(0) I3(1) I3(2) I3(3) I3(4) I3(5) I3(6) I3(7))
    } else if constexpr (K == 4) {  // v_add_f32
#define I4(j) asm volatile("v_add_f32 %0, %0, %1" : "+v"(s[j]) : "v"(sc));
      REP16(I4(0) I4(1) I4(2) I4(3) I4(4) I4(5) I4(6) I4(7))
    } else if constexpr (K == 5) {  // v_rcp_f32
#define I5(j) asm volatile("v_rcp_f32 %0, %0" : "+v"(s[j]));
      REP16(I5(0) I5(1) I5(2) I5(3) I5(4) I5(5) I5(6) I5(7))
    } else if constexpr (K == 6) {  // v_fma_f32 and v_pk_fma_f32 alternating
#define I6(j) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s[j]) : "v"(sb), "v"(sc)); \
              asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
      REP16(I6(0) I6(1) I6(2) I6(3)) REP16(I6(4) I6(5) I6(6) I6(7))
    } else if constexpr (K == 7) {  // v_fma_f32, one dependent chain
#define I7(j) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s[0]) : "v"(sb), "v"(sc));
      REP16(I7(0) I7(1) I7(2) I7(3) I7(4) I7(5) I7(6) I7(7))
    } else if constexpr (K == 8) {  // v_pk_fma_f32, one dependent chain
#define I8(j) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[0]) : "v"(b), "v"(c));
      REP16(I8(0) I8(1) I8(2) I8(3) I8(4) I8(5) I8(6) I8(7))
    } else if constexpr (K == 9) {  // v_mov_b32 + DPP row_shr:1 (the team reductions' form)
#define I9(j) asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(s[j]));
      REP16(I9(0) I9(1) I9(2) I9(3) I9(4) I9(5) I9(6) I9(7))
    } else if constexpr (K == 10) {  // v_add_f32 with a DPP operand
#define I10(j) asm volatile("v_add_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(s[j]) : "v"(sc));
      REP16(I10(0) I10(1) I10(2) I10(3) I10(4) I10(5) I10(6) I10(7))
    } else if constexpr (K == 11) {  // v_fmac_f32 (VOP2)
#define I11(j) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(s[j]) : "v"(sb), "v"(sc));
      REP16(I11(0) I11(1) I11(2) I11(3) I11(4) I11(5) I11(6) I11(7))
    } else if constexpr (K == 12) {  // v_fmac_f32 with a 32-bit literal operand (the SAT's hull constants)
#define I12(j) asm volatile("v_fmac_f32 %0, 0x3f8ccccd, %1" : "+v"(s[j]) : "v"(sc));
      REP16(I12(0) I12(1) I12(2) I12(3) I12(4) I12(5) I12(6) I12(7))
    } else if constexpr (K == 13) {  // s_mov_b32 literal + v_pk_fma_f32 with that SGPR splat (per pair, 2 instr)
#define I13(j) asm volatile("s_mov_b32 s90, 0x3f8ccccd\n v_pk_fma_f32 %0, %0, s[90:91], %1 op_sel_hi:[1,0,1]" : "+v"(a[j]) : "v"(c) : "s90", "s91");
      REP16(I13(0) I13(1) I13(2) I13(3) I13(4) I13(5) I13(6) I13(7))
    } else if constexpr (K == 14) {  // v_pk_fma_f32 with an inline-constant splat
#define I14(j) asm volatile("v_pk_fma_f32 %0, %0, 0.5, %1 op_sel_hi:[1,0,1]" : "+v"(a[j]) : "v"(c));
      REP16(I14(0) I14(1) I14(2) I14(3) I14(4) I14(5) I14(6) I14(7))
    } else if constexpr (K == 15) {  // v_cndmask_b32 (the SAT's selects)
#define I15(j) asm volatile("v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(s[j]) : "v"(sc) : "vcc");
      REP16(I15(0) I15(1) I15(2) I15(3) I15(4) I15(5) I15(6) I15(7))
    } else if constexpr (K == 16) {  // v_max3_f32 / v_min3_f32
#define I16(j) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(s[j]) : "v"(sb), "v"(sc));
      REP16(I16(0) I16(1) I16(2) I16(3) I16(4) I16(5) I16(6) I16(7))
    }
  }
  const long long t1 = clock64();
  float acc = 0.0f;
  for (int i = 0; i < 8; i++) acc += s[i] + a[i].x + a[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int K>
static double run(float* out, long long* cyc_d, long long* cyc_h, int nb, int iters) {
  hipLaunchKernelGGL(probe<K>, dim3(nb), dim3(256), 0, 0, out, cyc_d, iters);
  hipLaunchKernelGGL(probe<K>, dim3(nb), dim3(256), 0, 0, out, cyc_d, iters);
  hipDeviceSynchronize();
  hipMemcpy(cyc_h, cyc_d, sizeof(long long) * nb * 4, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < nb * 4; i++) s += (double)cyc_h[i];
  return s / (nb * 4) / (iters * 128.0);
}

int main() {
  const int nb = 256, iters = 2000;
  float* out;
  long long *cyc_d, cyc_h[nb * 4];
  hipMalloc(&out, sizeof(float) * nb * 256);
  hipMalloc(&cyc_d, sizeof(long long) * nb * 4);
  const char* names[] = {"v_fma_f32 x8 chains", "v_pk_fma_f32 x8 chains", "v_pk_mul_f32 x8", "v_pk_add_f32 x8",
                         "v_add_f32 x8", "v_rcp_f32 x8", "v_fma_f32 + v_pk_fma_f32 alternating (per pair)",
                         "v_fma_f32 dependent chain", "v_pk_fma_f32 dependent chain", "v_mov_b32_dpp row_shr x8",
                         "v_add_f32_dpp row_shr x8", "v_fmac_f32 x8", "v_fmac_f32 literal x8",
                         "s_mov_b32 literal + v_pk_fma_f32 sgpr splat (per pair)", "v_pk_fma_f32 inline-constant splat",
                         "v_cmp + v_cndmask (per pair)", "v_max3_f32"};
  double r[17];
  r[0] = run<0>(out, cyc_d, cyc_h, nb, iters);
  r[1] = run<1>(out, cyc_d, cyc_h, nb, iters);
  r[2] = run<2>(out, cyc_d, cyc_h, nb, iters);
  r[3] = run<3>(out, cyc_d, cyc_h, nb, iters);
  r[4] = run<4>(out, cyc_d, cyc_h, nb, iters);
  r[5] = run<5>(out, cyc_d, cyc_h, nb, iters);
  r[6] = run<6>(out, cyc_d, cyc_h, nb, iters);
  r[7] = run<7>(out, cyc_d, cyc_h, nb, iters);
  r[8] = run<8>(out, cyc_d, cyc_h, nb, iters);
  r[9] = run<9>(out, cyc_d, cyc_h, nb, iters);
  r[10] = run<10>(out, cyc_d, cyc_h, nb, iters);
  r[11] = run<11>(out, cyc_d, cyc_h, nb, iters);
  r[12] = run<12>(out, cyc_d, cyc_h, nb, iters);
  r[13] = run<13>(out, cyc_d, cyc_h, nb, iters);
  r[14] = run<14>(out, cyc_d, cyc_h, nb, iters);
  r[15] = run<15>(out, cyc_d, cyc_h, nb, iters);
  r[16] = run<16>(out, cyc_d, cyc_h, nb, iters);
  printf("one wave per SIMD, %d workgroups x 256 threads, s_memtime cycles per wave-instruction:\n", nb);
  for (int k = 0; k < 17; k++) printf("  %-52s %.2f\n", names[k], r[k]);
  hipError_t e = hipGetLastError();
  printf("status: %s\n", hipGetErrorString(e));
  return e == hipSuccess ? 0 : 1;
}
