// duck_team.h — mjx.step with a team of 16 lanes per env (CDNA4, fp32).
//
// Same physics, same LDS layout (Lay<Md>) and same arithmetic as duck_physics.h, but each
// env is worked by 16 consecutive lanes of a wave (4 envs per wave, 4 waves per CU at
// 16 envs per CU): lanes split every stage's independent items — bodies of one tree level,
// degrees of freedom, mass-matrix entries, LDL' updates of one pivot, hull vertices,
// constraint rows — and combine with DPP row reductions. A team never spans waves, so a
// team barrier is only a compiler ordering point (LDS operations of one wave complete in
// issue order).
//
// The env slice is contiguous (element k of env t at lds[t*STRIDE + k]); STRIDE = 16 mod 32
// so the two teams of a 32-lane half hit disjoint banks. The rare foot/foot contact runs its
// hull/hull SAT and dense Newton direction team-parallel too, out of line (collide_hulls_rare,
// newton_dense).
#pragma once
#include <utility>

#include "duck_physics.h"

constexpr int TEAM = 16;
constexpr int TEAM_WG = 16;  // envs (teams) per workgroup: 256 threads = 4 waves
constexpr int TPB_TEAM = TEAM * TEAM_WG;
typedef __attribute__((address_space(3))) int lds_int;
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) f4v lds_f4;

// fp32 reciprocal as one v_rcp_f32 (1 ulp; operands here are never denormal or zero)
DK float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
// m's lane bit ? t : f, as one v_cndmask the compiler cannot turn back into an indexed load
DK float vsel(unsigned long long m, float t, float f) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
  return r;
}

// impedance of a constraint at violation pos (mjx constraint._kbi, imp part)
DK float imp_of(const float* solimp, float pos) {
  const float dmin = fminf(fmaxf(solimp[0], 0.0001f), 0.9999f), dmax = fminf(fmaxf(solimp[1], 0.0001f), 0.9999f);
  const float width = fmaxf(1e-15f, solimp[2]), mid = fminf(fmaxf(solimp[3], 0.0001f), 0.9999f);
  const float power = fmaxf(1.0f, solimp[4]);
  const float x = fabsf(pos) * frcp(width);
  float y;
  if (power == 2.0f) {
    y = x < mid ? frcp(mid) * x * x : 1.0f - frcp(1.0f - mid) * (1.0f - x) * (1.0f - x);
  } else {
    y = x < mid ? (1.0f / powf(mid, power - 1.0f)) * powf(x, power)
                : 1.0f - (1.0f / powf(1.0f - mid, power - 1.0f)) * powf(1.0f - x, power);
  }
  const float im = fminf(fmaxf(dmin + y * (dmax - dmin), dmin), dmax);
  return x > 1.0f ? dmax : im;
}

#define TSYNC()                           \
  do {                                    \
    asm volatile("" ::: "memory");        \
    __builtin_amdgcn_wave_barrier();      \
    asm volatile("" ::: "memory");        \
  } while (0)

// DPP reads with every lane of the row valid (full masks): no "old" value is needed, so the
// mov has an undefined old operand and folds into its consumer (v_add_f32_dpp, v_mul_f32_dpp)
// without a zeroing v_mov per read
template <int CTRL>
DK float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
DK int dppi(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}
// min / max without the v_max_f32 x, x, x (canonicalize) that the compiler puts in front of fminf /
// fmaxf for each operand it cannot prove canonical -- a DPP read, an output of a multi-result asm
// statement: v_med3 with an infinite third operand (one instruction; a DPP read stays a separate
// v_mov_b32_dpp, VOP3 has no DPP form here). Same results for every non-NaN operand
// (the infinity opaque: with a constant one the compiler rewrites v_med3 as fminf / fmaxf again)
DK float fmin_nc(float a, float b) {
  float ninf = -__builtin_inff();
  asm("" : "+s"(ninf));
  return __builtin_amdgcn_fmed3f(a, b, ninf);
}
DK float fmax_nc(float a, float b) {
  float inf = __builtin_inff();
  asm("" : "+s"(inf));
  return __builtin_amdgcn_fmed3f(a, b, inf);
}
// reductions over the 16 lanes of a DPP row (= one team); every lane gets the result
DK float tsum(float v) {
  v += dppf<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dppf<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dppf<0x141>(v);  // row_half_mirror
  v += dppf<0x140>(v);  // row_mirror
  return v;
}
// for (i = lane; i < N; i += TEAM) f(i), the trip count unrolled at compile time: straight-line code
// instead of a loop whose trip count depends on the lane (exec-masked loop control per iteration)
template <int N, int B0 = 0, class F>
DK void team_for(int lane, F&& f) {
#pragma unroll
  for (int s = 0; s < (N - B0 + TEAM - 1) / TEAM; s++) {
    const int i = B0 + lane + TEAM * s;
    if (B0 + TEAM * (s + 1) <= N || i < N) f(i);
  }
}
DK float tmaxf(float v) {
  v = fmaxf(v, dppf<0xB1>(v));
  v = fmaxf(v, dppf<0x4E>(v));
  v = fmaxf(v, dppf<0x141>(v));
  v = fmaxf(v, dppf<0x140>(v));
  return v;
}
DK int tmini(int v) {
  v = min(v, dppi<0xB1>(v));
  v = min(v, dppi<0x4E>(v));
  v = min(v, dppi<0x141>(v));
  v = min(v, dppi<0x140>(v));
  return v;
}
// reductions over the 8-lane halves of a team
DK float hsum8(float v) {
  v += dppf<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dppf<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dppf<0x141>(v);  // row_half_mirror
  return v;
}
DK float hmax8(float v) {
  v = fmaxf(v, dppf<0xB1>(v));
  v = fmaxf(v, dppf<0x4E>(v));
  v = fmaxf(v, dppf<0x141>(v));
  return v;
}
// the same with fmax_nc (the height field's reductions: C4 / C5 +0.4-0.6 %; in the flat scenes'
// plane contacts the med3 form measured 0.4 % slower, C2)
DK float hmax8_nc(float v) {
  v = fmax_nc(v, dppf<0xB1>(v));
  v = fmax_nc(v, dppf<0x4E>(v));
  v = fmax_nc(v, dppf<0x141>(v));
  return v;
}
DK int hmin8i(int v) {
  v = min(v, dppi<0xB1>(v));
  v = min(v, dppi<0x4E>(v));
  v = min(v, dppi<0x141>(v));
  return v;
}

// Compile-time loops and compile-time vectors as instruction literals. The height field's SAT
// multiplies per-lane vectors by hundreds of hull constants (face normals, edge directions,
// vertices), each used several times: the compiler keeps such a constant in an SGPR, and with
// this many the SGPRs spill to VGPR lanes (one v_readlane per use, 20 % of the SAT's
// instructions). As a 32-bit literal of a VOP2 multiply / multiply-add it costs nothing.
template <int B, int E, class F>
DK void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}
constexpr int fbits(float v) { return __builtin_bit_cast(int, v); }
// c . x for c = (C0, C1, C2) (float bit patterns)
template <int C0, int C1, int C2>
DK float cdot(const float* x) {
  float r;
  asm("v_mul_f32_e32 %0, %1, %2" : "=v"(r) : "i"(C0), "v"(x[0]));
  asm("v_fmac_f32_e32 %0, %1, %2" : "+v"(r) : "i"(C1), "v"(x[1]));
  asm("v_fmac_f32_e32 %0, %1, %2" : "+v"(r) : "i"(C2), "v"(x[2]));
  return r;
}
// c . x, c . y, c . z, c . u (and c . w): the same products as cdot, interleaved in one statement.
// The scheduler prices an asm statement at no latency, so separate per-instruction statements were
// left as dependent mul -> fmac -> fmac chains, each link stalled (8 cycles for one wave, against 4-5
// independent) and padded with an s_nop that the hazard recognizer puts after inline asm
// OFF - c . x, OFF - c . y, OFF - c . z: three products and the subtraction in one statement
template <int C0, int C1, int C2, int OFF>
DK void cdot3v_off(const float* x, const float* y, const float* z, float* r) {
  asm("v_mul_f32_e32 %0, %3, %7\n\tv_mul_f32_e32 %1, %3, %10\n\tv_mul_f32_e32 %2, %3, %13\n\t"
      "v_fmac_f32_e32 %0, %4, %8\n\tv_fmac_f32_e32 %1, %4, %11\n\tv_fmac_f32_e32 %2, %4, %14\n\t"
      "v_fmac_f32_e32 %0, %5, %9\n\tv_fmac_f32_e32 %1, %5, %12\n\tv_fmac_f32_e32 %2, %5, %15\n\t"
      "v_sub_f32_e32 %0, %6, %0\n\tv_sub_f32_e32 %1, %6, %1\n\tv_sub_f32_e32 %2, %6, %2"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2])
      : "i"(C0), "i"(C1), "i"(C2), "i"(OFF), "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(y[0]), "v"(y[1]), "v"(y[2]),
        "v"(z[0]), "v"(z[1]), "v"(z[2]));
}
template <int C0, int C1, int C2>
DK void cdot4v(const float* x, const float* y, const float* z, const float* u, float* r) {
  asm("v_mul_f32_e32 %0, %4, %7\n\tv_mul_f32_e32 %1, %4, %10\n\tv_mul_f32_e32 %2, %4, %13\n\t"
      "v_mul_f32_e32 %3, %4, %16\n\t"
      "v_fmac_f32_e32 %0, %5, %8\n\tv_fmac_f32_e32 %1, %5, %11\n\tv_fmac_f32_e32 %2, %5, %14\n\t"
      "v_fmac_f32_e32 %3, %5, %17\n\t"
      "v_fmac_f32_e32 %0, %6, %9\n\tv_fmac_f32_e32 %1, %6, %12\n\tv_fmac_f32_e32 %2, %6, %15\n\t"
      "v_fmac_f32_e32 %3, %6, %18"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3])
      : "i"(C0), "i"(C1), "i"(C2), "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(y[0]), "v"(y[1]), "v"(y[2]),
        "v"(z[0]), "v"(z[1]), "v"(z[2]), "v"(u[0]), "v"(u[1]), "v"(u[2]));
}
template <int C0, int C1, int C2>
DK void cdot5v(const float* x, const float* y, const float* z, const float* u, const float* w, float* r) {
  asm("v_mul_f32_e32 %0, %5, %8\n\tv_mul_f32_e32 %1, %5, %11\n\tv_mul_f32_e32 %2, %5, %14\n\t"
      "v_mul_f32_e32 %3, %5, %17\n\tv_mul_f32_e32 %4, %5, %20\n\t"
      "v_fmac_f32_e32 %0, %6, %9\n\tv_fmac_f32_e32 %1, %6, %12\n\tv_fmac_f32_e32 %2, %6, %15\n\t"
      "v_fmac_f32_e32 %3, %6, %18\n\tv_fmac_f32_e32 %4, %6, %21\n\t"
      "v_fmac_f32_e32 %0, %7, %10\n\tv_fmac_f32_e32 %1, %7, %13\n\tv_fmac_f32_e32 %2, %7, %16\n\t"
      "v_fmac_f32_e32 %3, %7, %19\n\tv_fmac_f32_e32 %4, %7, %22"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4])
      : "i"(C0), "i"(C1), "i"(C2), "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(y[0]), "v"(y[1]), "v"(y[2]),
        "v"(z[0]), "v"(z[1]), "v"(z[2]), "v"(u[0]), "v"(u[1]), "v"(u[2]), "v"(w[0]), "v"(w[1]), "v"(w[2]));
}
// o_i - c . x_i for the five vectors x, y, z, u, w and per-lane offsets o: the first product fused
// with its offset (v_fmamk_f32: literal -c_0, no separate subtraction)
template <int C0, int C1, int C2>
DK void cdot5v_noff(const float* x, const float* y, const float* z, const float* u, const float* w, const float* o,
                    float* r) {
  asm("v_fmamk_f32 %0, %8, %5, %23\n\tv_fmamk_f32 %1, %11, %5, %24\n\tv_fmamk_f32 %2, %14, %5, %25\n\t"
      "v_fmamk_f32 %3, %17, %5, %26\n\tv_fmamk_f32 %4, %20, %5, %27\n\t"
      "v_fmac_f32_e32 %0, %6, %9\n\tv_fmac_f32_e32 %1, %6, %12\n\tv_fmac_f32_e32 %2, %6, %15\n\t"
      "v_fmac_f32_e32 %3, %6, %18\n\tv_fmac_f32_e32 %4, %6, %21\n\t"
      "v_fmac_f32_e32 %0, %7, %10\n\tv_fmac_f32_e32 %1, %7, %13\n\tv_fmac_f32_e32 %2, %7, %16\n\t"
      "v_fmac_f32_e32 %3, %7, %19\n\tv_fmac_f32_e32 %4, %7, %22"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4])
      : "i"(C0 ^ (int)0x80000000), "i"(C1 ^ (int)0x80000000), "i"(C2 ^ (int)0x80000000), "v"(x[0]), "v"(x[1]),
        "v"(x[2]), "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(z[0]), "v"(z[1]), "v"(z[2]), "v"(u[0]), "v"(u[1]), "v"(u[2]),
        "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]), "v"(o[4]));
}
// a . x and b . x for two compile-time vectors a = (A0, A1, A2), b = (B0, B1, B2), interleaved
template <int A0, int A1, int A2, int B0, int B1, int B2>
DK void cdot2c(const float* x, float& ra, float& rb) {
  asm("v_mul_f32_e32 %0, %2, %8\n\tv_mul_f32_e32 %1, %5, %8\n\t"
      "v_fmac_f32_e32 %0, %3, %9\n\tv_fmac_f32_e32 %1, %6, %9\n\t"
      "v_fmac_f32_e32 %0, %4, %10\n\tv_fmac_f32_e32 %1, %7, %10"
      : "=&v"(ra), "=&v"(rb)
      : "i"(A0), "i"(A1), "i"(A2), "i"(B0), "i"(B1), "i"(B2), "v"(x[0]), "v"(x[1]), "v"(x[2]));
}
// a + c * x (fma with a literal c)
template <int C>
DK float cfma(float x, float a) {
  asm("v_fmac_f32_e32 %0, %1, %2" : "+v"(a) : "i"(C), "v"(x));
  return a;
}

// the height field's contact point when no vertex of either shape is inside the other: the
// support features' vertices within this band (m) of the support plane (oracle HF_WITNESS_BAND)
constexpr float HF_WITNESS_BAND = 1e-3f;
// depths within this (m) of the deepest prism contact count as equal (oracle HF_DEPTH_TIE)
constexpr float HF_DEPTH_TIE = 1e-6f;

#ifndef DUCK_LS_DFLOOR
#define DUCK_LS_DFLOOR 1e-6f
#endif

// Latency mode (LAT, step_kernel_lat): the stages of one substep are split over the four waves of a
// workgroup that all work the same 4 envs (wave 0: kinematics, com_pos, rne, actuation and the env
// code; wave 1: composite inertias, crb, the warm start, the Newton solve, sensors, Euler; wave 2:
// collision and the constraint rows; wave 3: M's factorization and the smooth solve). Waves that run concurrently must not
// share scratch, so a latency slice gives rne's scratch, the composite inertias and the height
// field's silhouette lists regions of their own after the throughput slice's words.
constexpr int LAT_WG = 4;  // envs (teams) per latency-mode workgroup: 4 waves x 4 teams, one team set per wave
// latency-mode event waits that gave up (TPhys::ev_wait; read by duck_debug_lat_timeouts, must stay 0)
static __device__ unsigned int g_lat_timeouts;
// -DDUCK_LAT_PROF (tools/lat_prof.py): clock64 of each cross-wave event of substep 5 in workgroup 0, into
// the per-wave cycle slots of g_stage_cycles (which only the throughput kernel writes)
#ifdef DUCK_LAT_PROF
#define LAT_T(k, s)                                                                                         \
  do {                                                                                                      \
    if (blockIdx.x == 0 && ((int)threadIdx.x & 63) == 0 && (s) == 5) g_stage_cycles[DUCK_NSTAGE + (k)] = clock64(); \
  } while (0)
#define LAT2_T(k, s)               \
  do {                             \
    if (threadIdx.x < 128) LAT_T(k, s); \
  } while (0)
#else
#define LAT_T(k, s) \
  do {              \
  } while (0)
#define LAT2_T(k, s) \
  do {               \
  } while (0)
#endif

// LAT: 0 = the throughput kernel (one team per env, 16 envs per workgroup); 1 = the latency kernel
// (4 envs per workgroup, each substep's stages over 4 waves); 2 = the paired latency kernel (8 envs per
// workgroup, each set of 4 envs on a pair of waves: the stages split over 2 waves)
template <class Md, int LAT = 0>
struct TLay {
  using Ly = Lay<Md>;
  // per-lane dump slots (SINK, 2 x TEAM words; debug line-search dumps use 136 words from here)
  static constexpr int KC = Ly::TOTAL;
#ifdef DUCK_LS_DUMP
  static constexpr int USED0 = KC + 136;
#else
  static constexpr int USED0 = KC + 2 * TEAM;
#endif
  // the height field's per-foot silhouette lists (collide_hfield -> hf_exec)
  static constexpr int HF_SLF = (1 + Md::HF_SILCAP + 3) & ~3;
  static constexpr int HF_SLSZ = HF_SLF + 4 * Md::HF_SILCAP;
  // rne's scratch: body accelerations (6 NB), subtree forces (6 NB), body forces (6 NB)
  static constexpr int XRNE = LAT ? ((USED0 + 3) & ~3) : Ly::H;
  static constexpr int RCA = XRNE, CFRC = XRNE + 6 * Md::NB, RFB = XRNE + 12 * Md::NB;
  // composite inertias (summed by rne's subtree pass, read by crb); throughput mode overwrites the
  // body inertias in CIN (phase B of rne has read them)
  static constexpr int XCIN = LAT ? XRNE + 18 * Md::NB : Ly::CIN;
  // the subtree pass's lanes that a latency-mode wave does not own write here (forces / inertias)
  static constexpr int XDUM0 = LAT ? XCIN + 10 * Md::NB : 0, XDUM1 = LAT ? XDUM0 + 10 * Md::NB : 0;
  static constexpr int XSIL = LAT ? ((XDUM1 + 6 * Md::NB + 3) & ~3) : ((Ly::CIN + 3) & ~3);
  // the speculative Newton direction of wave 3 (latency mode): NV floats, then the team's valid flag
  static constexpr int XDIR = LAT ? ((XSIL + (Md::FLOOR_TYPE == 1 ? 2 * HF_SLSZ : 0) + 3) & ~3) : 0;
  static constexpr int USED = LAT ? XDIR + Md::NV + 4 : USED0;
  static constexpr int STRIDE = ((USED + 15) / 32) * 32 + 16;  // = 16 (mod 32), >= USED
  static constexpr int NWG = LAT == 2 ? 2 * LAT_WG : (LAT ? LAT_WG : TEAM_WG);  // envs per workgroup
  static_assert(STRIDE >= USED && STRIDE % 32 == 16, "stride");
  // per-lane dump slots for branchless conditional stores (L[ok ? addr : SINK + lane] = v): a
  // lane-divergent `if` leaves a join block whose exec restore the register allocator may put
  // live-range split copies in front of (tools/isa_exec_check.py), so the hot
  // path avoids such regions where a select does the job.
  static constexpr int SINK = KC;
  // scratch of the flattened tree passes: the H + constraint-row storage is dead until the
  // constraint stage (kinematics / rne / crb run before it)
  static constexpr int TMP = Ly::H;
  static constexpr int KLOC = TMP;                               // local body transforms (7 per body)
  static_assert(7 * Md::NB <= Ly::HSZ + 4 * Ly::NROW, "tree scratch must fit in H + rows");
  // the model blob (lane-indexed tables, constraint-row records) follows the env slices in
  // LDS when it fits, else it is read from global memory
  static constexpr int TAB = STRIDE * NWG;
  // step_kernel stages each env's hot state (the duck_layout fields before first_qpos) in LDS:
  // one batch of independent global loads in, one batch of stores out
  static constexpr int HOT = Md::NQ + 2 * Md::NV + 8 * Md::NU + 77;
  static constexpr int ESTRIDE = (HOT + 64) | 1;  // + the step's 64 random draws; odd: distinct banks
  static constexpr int ES_FLOATS = ESTRIDE * NWG;
  // latency modes: the cross-wave event counters, one 16-B word group each, in front of the slices'
  // end of LDS (LDS_FLOATS counts them); NEV_G per set of 4 envs (the paired kernel has two sets)
  static constexpr int NEV_G = LAT ? 10 : 0;
  static constexpr int NEV = LAT == 2 ? 2 * NEV_G : NEV_G;
  static constexpr size_t LDS_MAX = 160 * 1024 / 4 - 4 * NEV;
  // LDS priority: model blob (read every substep), then the hot state (read once per env-step)
  static constexpr bool TAB_LDS = (size_t)(TAB + Md::NBLOB) <= LDS_MAX;
  // the height field's hull SAT tables (hull faces + edges, contiguous in the blob) in LDS on their
  // own when the whole blob is not (rough + backlash: the prism loop reads them per prism)
  static constexpr int NHT = Md::B_HEND > Md::B_HFACE ? Md::B_HEND - Md::B_HFACE : 0;
  static constexpr bool HT_LDS = !TAB_LDS && NHT > 0 && (size_t)(TAB + NHT) <= LDS_MAX;
  static constexpr int ES = TAB + (TAB_LDS ? Md::NBLOB : (HT_LDS ? NHT : 0));
  static constexpr bool ES_LDS = (size_t)(ES + ES_FLOATS) <= LDS_MAX;
  static constexpr int EV = ES + (ES_LDS ? ES_FLOATS : 0);
  static constexpr int LDS_FLOATS = EV + 4 * NEV;
  // whether this work split can run the model at all: the throughput kernel needs its env slices in
  // LDS; the latency kernels also need the model blob and the hot state there (step_kernel_lat). A
  // model that fits the throughput kernel but not a latency split compiles without that split
  // (duck_env_kernels.h launch_step; AUTO then falls back, duck_set_step_mode refuses it)
  static constexpr bool FITS = (size_t)LDS_FLOATS * 4 <= 160 * 1024 && (LAT == 0 || (TAB_LDS && ES_LDS));
  static_assert(LAT || FITS, "LDS budget");
  static_assert(6 * Md::NV <= 4 * Ly::NROW, "crb scratch must fit in the row storage");
  static_assert(LAT || 18 * Md::NB <= Ly::HSZ + 4 * Ly::NROW, "rne scratch must fit in H + rows");
  static_assert(LAT || Md::FLOOR_TYPE != 1 || XSIL + 2 * HF_SLSZ <= Ly::CIN + 10 * Md::NB,
                "the silhouette lists must fit in the composite inertias' storage");
};

// copy the model blob into the workgroup's LDS (before any thread of the block exits)
template <class Md, int LAT = 0>
DK void load_model_tables(float* lds) {
  using TLy = TLay<Md, LAT>;
  if constexpr (TLy::TAB_LDS) {
    // a compile-time trip count: every load of the thread is issued before the first store waits
    // (a runtime-bounded loop waits for each group of loads: one memory round trip per group)
    int* dst = (int*)(lds + TLy::TAB);
    constexpr int NK = (Md::NBLOB + TPB_TEAM - 1) / TPB_TEAM;
    int w[NK];
#pragma unroll
    for (int kk = 0; kk < NK; kk++) {
      const int i = (int)threadIdx.x + TPB_TEAM * kk;
      w[kk] = Md::t_blob()[i < Md::NBLOB ? i : Md::NBLOB - 1];
    }
#pragma unroll
    for (int kk = 0; kk < NK; kk++) {
      const int i = (int)threadIdx.x + TPB_TEAM * kk;
      if (i < Md::NBLOB) dst[i] = w[kk];
    }
    __syncthreads();
  } else if constexpr (TLy::HT_LDS) {
    int* dst = (int*)(lds + TLy::TAB);
    constexpr int N = TLy::NHT, NK = (N + TPB_TEAM - 1) / TPB_TEAM;
    int w[NK];
#pragma unroll
    for (int kk = 0; kk < NK; kk++) {
      const int i = (int)threadIdx.x + TPB_TEAM * kk;
      w[kk] = Md::t_blob()[Md::B_HFACE + (i < N ? i : N - 1)];
    }
#pragma unroll
    for (int kk = 0; kk < NK; kk++) {
      const int i = (int)threadIdx.x + TPB_TEAM * kk;
      if (i < N) dst[i] = w[kk];
    }
    __syncthreads();
  }
}

// the hull's faces in screening order for the prism-vertex-inside-hull test (hf_exec): the six faces
// whose normals are extreme along -z, +z, +x, -x, +y, -y of the mesh frame first (a grid vertex near
// a foot is almost always outside one of them: below the sole, above the top or beside the
// footprint), then the rest in index order. The minimum over the faces does not depend on the order.
template <class Md>
struct HullFaceOrder {
  int f[Md::NHF];
  constexpr HullFaceOrder() : f{} {
    bool used[Md::NHF] = {};
    int n = 0;
    for (int c = 0; c < 6 && c < Md::NHF; c++) {
      const int ax = c < 2 ? 2 : (c < 4 ? 0 : 1);
      const float sg = (c == 0 || c == 3 || c == 5) ? -1.0f : 1.0f;
      int best = -1;
      for (int i = 0; i < Md::NHF; i++)
        if (!used[i] && (best < 0 || sg * Md::hull_face_normal[i][ax] > sg * Md::hull_face_normal[best][ax])) best = i;
      used[best] = true;
      f[n++] = best;
    }
    for (int i = 0; i < Md::NHF; i++)
      if (!used[i]) f[n++] = i;
  }
};

template <class Md, int LAT = 0>
struct TPhys {
  using Ly = Lay<Md>;
  using TL = TLay<Md, LAT>;
  using P1 = Phys<Md, 1>;
  using S1 = Slice<1>;
  typedef lds_float* LP;
  static constexpr int NV = Md::NV, NB = Md::NB, NQ = Md::NQ, NU = Md::NU, NJ = Md::NJ;
  static constexpr int NCON = Ly::NCON, NFRIC = Md::NFRIC, NLIM = Md::NLIM, NROW = Ly::NROW;
  static constexpr int R_LIM = Ly::R_LIM, R_CON = Ly::R_CON;
  static DK int ti(int off) {
    if constexpr (TL::TAB_LDS) {
      extern __shared__ float lds_dyn[];
      return ((lds_int*)(lds_dyn + TL::TAB))[off];
    } else {
      return Md::t_blob()[off];
    }
  }
  static DK float tf(int off) { return __int_as_float(ti(off)); }
  // the hull SAT tables (blob words B_HFACE .. B_HEND): LDS whenever they fit
  static DK float th(int off) {
    if constexpr (!TL::TAB_LDS && TL::HT_LDS) {
      extern __shared__ float lds_dyn[];
      return ((lds_float*)(lds_dyn + TL::TAB))[off - Md::B_HFACE];
    } else {
      return tf(off);
    }
  }
  // a 16-B record of the hull SAT tables (blob words B_HFACE .. B_HEND, 16-B aligned, in LDS for
  // the height-field scenes): the reads indexed per lane (the unrolled loops over all faces and
  // edges take the compile-time constants instead: as LDS reads they were 28 % slower)
  static DK f4v ht4(int off) {
    extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
    static_assert(Md::FLOOR_TYPE != 1 || TL::TAB_LDS || TL::HT_LDS, "the hull SAT tables must be in LDS");
    return *(const lds_f4*)((lds_float*)lds_dyn + TL::TAB + (TL::TAB_LDS ? off : off - Md::B_HFACE));
  }
  static constexpr int LIMW = 13, PAIRW = 13;
  // row -> dof and dof -> row maps of the friction and limit rows: affine when the rows cover
  // consecutive dofs (codegen B_FRIC0 / B_LIM0 >= 0), else index words of the model blob
  static DK int fric_dof(int r) {
    if constexpr (Md::B_FRIC0 >= 0) return Md::B_FRIC0 + r;
    else return ti(Md::B_FRIC + 3 * r);
  }
  static DK int lim_dof(int r) {
    if constexpr (Md::B_LIM0 >= 0) return Md::B_LIM0 + r;
    else return ti(Md::B_LIM + LIMW * r);
  }
  static DK int dof_fric(int c) {
    if constexpr (Md::B_FRIC0 >= 0) return (c >= Md::B_FRIC0 && c < Md::B_FRIC0 + NFRIC) ? c - Md::B_FRIC0 : -1;
    else return ti(Md::B_DOF2FRIC + c);
  }
  static DK int dof_lim(int c) {
    if constexpr (Md::B_LIM0 >= 0) return (c >= Md::B_LIM0 && c < Md::B_LIM0 + NLIM) ? c - Md::B_LIM0 : -1;
    else return ti(Md::B_DOF2LIM + c);
  }
  static DK int madr(int i, int j) { return ti(Md::B_MADR + NV * i + j); }
  // lane-indexed model constants live in the LDS blob (codegen.team_tables records)
  // dofs 0-2 are the translational dofs of the trunk's free joint: their motion axes (cdof rows,
  // com_pos) are the unit vectors e_3, e_4, e_5, so cdof_i . x = x[3 + i] exactly for i < 3 and the
  // products that read those rows are skipped
  static constexpr bool FREE0 = Md::jnt_type[0] == 0 && Md::body_dofadr[1] == 0 && Md::body_dofnum[1] == 6;
  static constexpr unsigned long long moving_mask() {
    unsigned long long msk = 0;
    for (int b = 0; b < Md::NB; b++)
      if (Md::body_weldid[b] != 0) msk |= 1ull << b;
    return msk;
  }
  static DK bool moving(int b) { return (moving_mask() >> b) & 1ull; }
  static DK int limb_body(int lane, int d) { return ti(Md::B_BR + Md::T_BRLEN * (lane < Md::T_NBR ? lane : 0) + d); }
  static DK int limb_dof(int lane, int k) { return ti(Md::B_BRDOF + 2 * Md::T_BRLEN * (lane < Md::T_NBR ? lane : 0) + k); }
  static DK int dof_body(int i) {
    if constexpr (Md::B_DBD > -1000) return i < Md::B_DBN ? Md::B_DB0 : i + Md::B_DBD;
    else return ti(Md::B_DOFREC + 4 * i);
  }
  static DK int act_dof(int a) {
    if constexpr (Md::B_ACTD0 >= 0) return Md::B_ACTD0 + a;
    else return ti(Md::B_ACT + 12 * a + 5);
  }
  static DK int act_qadr(int a) {
    if constexpr (Md::B_ACTQ0 >= 0) return Md::B_ACTQ0 + a;
    else return ti(Md::B_ACT + 12 * a + 4);
  }
  static DK int lim_qadr(int r) {
    if constexpr (Md::B_LIMQ0 >= 0) return Md::B_LIMQ0 + r;
    else return ti(Md::B_LIM + LIMW * r + 1);
  }

  static_assert(NFRIC <= TEAM, "one friction row per lane");
  static_assert(NCON <= TEAM, "one contact slot per lane");
  static_assert(NU <= TEAM, "one actuator per lane");

  // ---------------- mj_kinematics: root path on every lane, one limb per lane ----------------
  // child pose from the parent pose held in registers
  static DK void body_pose(LP L, int b, const float* pp, const float* pR, const float* pq, float* p, float* q,
                           float* R) {
    const float bq[4] = {Md::body_quat[b][0], Md::body_quat[b][1], Md::body_quat[b][2], Md::body_quat[b][3]};
    const float bp[3] = {Md::body_pos[b][0], Md::body_pos[b][1], Md::body_pos[b][2]};
    float t[3];
    mulmv3(t, pR, bp);
    for (int k = 0; k < 3; k++) p[k] = pp[k] + t[k];
    qmul(q, pq, bq);
    const int nj = Md::body_jntnum[b], j0 = Md::body_jntadr[b];
#pragma unroll
    for (int jj = 0; jj < 2; jj++) {
      if (jj < nj) {
        const int j = j0 + jj, a = Md::jnt_qposadr[j];
        float sn, cs;
        sincosf(0.5f * (L[Ly::QPOS + a] - L[Ly::DQ0 + a]), &sn, &cs);
        const float ql[4] = {cs, Md::jnt_axis[j][0] * sn, Md::jnt_axis[j][1] * sn, Md::jnt_axis[j][2] * sn};
        qmul(q, q, ql);
      }
    }
    qnormalize(q);
    q2m(R, q);
  }
  static DK void store_pose(LP L, int b, const float* p, const float* q, const float* R) {
    for (int k = 0; k < 3; k++) L[Ly::XPOS + 3 * b + k] = p[k];
    for (int k = 0; k < 4; k++) L[Ly::XQ + 4 * b + k] = q[k];
    for (int k = 0; k < 9; k++) L[Ly::XMAT + 9 * b + k] = R[k];
  }

  static DK void kinematics(LP L, int lane) {
#pragma clang fp reassociate(on)
    STAGE_T0();
    // K1: local transform (body quat x joint rotations, body pos) of every moving body, a
    // body per lane, off the serial chain
    team_for<NB, 2>(lane, [&](int b) {
      if (!moving(b)) return;
      const int o = Md::B_BKIN + 17 * b;
      float q[4] = {tf(o), tf(o + 1), tf(o + 2), tf(o + 3)};
      const int nj = ti(o + 7);
#pragma unroll
      for (int jj = 0; jj < 2; jj++) {
        if (jj < nj) {
          const int oj = o + 8 + 4 * jj, a = ti(oj);
          float sn, cs;
          __sincosf(0.5f * (L[Ly::QPOS + a] - L[Ly::DQ0 + a]), &sn, &cs);
          const float ql[4] = {cs, tf(oj + 1) * sn, tf(oj + 2) * sn, tf(oj + 3) * sn};
          qmul(q, q, ql);
        }
      }
      for (int k = 0; k < 4; k++) L[TL::KLOC + 7 * b + k] = q[k];
      for (int k = 0; k < 3; k++) L[TL::KLOC + 7 * b + 4 + k] = tf(o + 4 + k);
    });
    TSYNC();
    STAGE_MARK(24);
    // K2: compose down the root path (every lane) and the limbs (a limb per lane)
    float p[3], q[4], R[9];
    for (int k = 0; k < 3; k++) p[k] = L[Ly::QPOS + k];
    for (int k = 0; k < 4; k++) q[k] = L[Ly::QPOS + 3 + k];
    qnormalize(q);
    q2m(R, q);
    if (lane == 0) store_pose(L, 1, p, q, R);
    auto compose = [&](int b) {
      float ql[4], pl[3], t[3], qn[4];
      for (int k = 0; k < 4; k++) ql[k] = L[TL::KLOC + 7 * b + k];
      for (int k = 0; k < 3; k++) pl[k] = L[TL::KLOC + 7 * b + 4 + k];
      mulmv3(t, R, pl);
      for (int k = 0; k < 3; k++) p[k] += t[k];
      qmul(qn, q, ql);
      qnormalize(qn);
      for (int k = 0; k < 4; k++) q[k] = qn[k];
      q2m(R, q);
    };
#pragma unroll
    for (int r = 1; r < Md::T_NROOT; r++) {
      compose(Md::T_ROOT[r]);
      if (lane == 0) store_pose(L, Md::T_ROOT[r], p, q, R);
    }
    if (lane < Md::T_NBR) {
      constexpr int BL = Md::T_BRLEN;
      int bb[BL];
      float kl[BL][7];  // the limb's local transforms, loaded before the chain (no LDS round trip per body)
#pragma unroll
      for (int d = 0; d < BL; d++) bb[d] = limb_body(lane, d);
#pragma unroll
      for (int d = 0; d < BL; d++) {
        const int bc = bb[d] >= 0 ? bb[d] : 1;
        for (int k = 0; k < 7; k++) kl[d][k] = L[TL::KLOC + 7 * bc + k];
      }
#pragma unroll
      for (int d = 0; d < BL; d++) {
        if (bb[d] < 0) break;
        float t[3], qn[4];
        mulmv3(t, R, &kl[d][4]);
        for (int k = 0; k < 3; k++) p[k] += t[k];
        qmul(qn, q, kl[d]);
        qnormalize(qn);
        for (int k = 0; k < 4; k++) q[k] = qn[k];
        q2m(R, q);
        store_pose(L, bb[d], p, q, R);
      }
    }
    TSYNC();
  }

  // ---------------- mj_comPos: subtree com (team reduction), cinert, cdof ----------------
  static DK void com_pos(LP L, int lane) {
#pragma clang fp reassociate(on)
    // every moving body fits the team (a body per lane): its inertial frame (xipos, the rotated
    // inertia) is formed once, held across the subtree-com reduction, and only the offset from the
    // com is applied after it
    static_assert((moving_mask() >> (1 + TEAM)) == 0, "a moving body per lane");
    float xi[3] = {0, 0, 0}, rot[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, m = 0.0f;
    const int b = 1 + lane;
    const bool mv = b < NB && moving(b);
    if (mv) {
      const int ob = Md::B_BINERT + 17 * b;
      float R[9], t[3], ip[3], Ri[9], Bi[9];
      for (int k = 0; k < 9; k++) R[k] = L[Ly::XMAT + 9 * b + k];
      for (int k = 0; k < 3; k++) ip[k] = (b == 1) ? L[Ly::DIPOS + k] : tf(ob + k);
      for (int k = 0; k < 9; k++) Bi[k] = tf(ob + 3 + k);
      mulmv3(t, R, ip);
      mulmm3(Ri, R, Bi);
      const float I[3] = {tf(ob + 12), tf(ob + 13), tf(ob + 14)};
      for (int a = 0; a < 3; a++)
        for (int c = 0; c < 3; c++)
          rot[3 * a + c] = Ri[3 * a] * I[0] * Ri[3 * c] + Ri[3 * a + 1] * I[1] * Ri[3 * c + 1] + Ri[3 * a + 2] * I[2] * Ri[3 * c + 2];
      for (int k = 0; k < 3; k++) xi[k] = L[Ly::XPOS + 3 * b + k] + t[k];
      m = L[Ly::DMASS + b];
    }
    const float ms = tsum(m);
    const float inv = frcp(ms);
    const float com[3] = {tsum(m * xi[0]) * inv, tsum(m * xi[1]) * inv, tsum(m * xi[2]) * inv};
    if (lane == 0)
      for (int k = 0; k < 3; k++) L[Ly::COM + k] = com[k];
    if (mv) {
      const float d[3] = {xi[0] - com[0], xi[1] - com[1], xi[2] - com[2]};
      const float dd = dot3(d, d);
      const int o = Ly::CIN + 10 * b;
      L[o + 0] = rot[0] + m * (dd - d[0] * d[0]);
      L[o + 1] = rot[4] + m * (dd - d[1] * d[1]);
      L[o + 2] = rot[8] + m * (dd - d[2] * d[2]);
      L[o + 3] = rot[1] - m * d[0] * d[1];
      L[o + 4] = rot[2] - m * d[0] * d[2];
      L[o + 5] = rot[5] - m * d[1] * d[2];
      L[o + 6] = m * d[0]; L[o + 7] = m * d[1]; L[o + 8] = m * d[2];
      L[o + 9] = m;
    }
    team_for<NJ>(lane, [&](int j) {
      const int oj = Md::B_JREC + 9 * j;
      // affine joint maps (codegen B_JAFF): hinge j >= B_JN0 sits on body j + B_JBD with dof j + B_JDD
      const bool jh = Md::B_JAFF && j >= Md::B_JN0;
      const int b = jh ? j + Md::B_JBD : ti(oj), da = jh ? j + Md::B_JDD : ti(oj + 1);
      const float off[3] = {com[0] - L[Ly::XPOS + 3 * b], com[1] - L[Ly::XPOS + 3 * b + 1], com[2] - L[Ly::XPOS + 3 * b + 2]};
      if (!jh && ti(oj + 3) == 0) {
        for (int k = 0; k < 3; k++)
          for (int q = 0; q < 6; q++) L[Ly::CDOF + 6 * (da + k) + q] = (q == 3 + k) ? 1.0f : 0.0f;
        for (int k = 0; k < 3; k++) {
          const float ax[3] = {L[Ly::XMAT + 9 * b + k], L[Ly::XMAT + 9 * b + 3 + k], L[Ly::XMAT + 9 * b + 6 + k]};
          float t[3];
          cross3(t, ax, off);
          const int o = Ly::CDOF + 6 * (da + 3 + k);
          L[o] = ax[0]; L[o + 1] = ax[1]; L[o + 2] = ax[2]; L[o + 3] = t[0]; L[o + 4] = t[1]; L[o + 5] = t[2];
        }
      } else {
        float R[9], ax[3], t[3];
        const float ja[3] = {tf(oj + 4), tf(oj + 5), tf(oj + 6)};
        for (int k = 0; k < 9; k++) R[k] = L[Ly::XMAT + 9 * b + k];
        mulmv3(ax, R, ja);
        cross3(t, ax, off);
        const int o = Ly::CDOF + 6 * da;
        L[o] = ax[0]; L[o + 1] = ax[1]; L[o + 2] = ax[2]; L[o + 3] = t[0]; L[o + 4] = t[1]; L[o + 5] = t[2];
      }
    });
    TSYNC();
  }

  // ---------------- mj_comVel + mj_rne (flg_acc = 0) ----------------
  // Three passes: (A) cvel/cacc down the tree — root path on every lane, a limb per lane, the
  // limb's cdof/qvel loaded into registers before the chain; (B) body forces
  // cinert cacc + cvel x* (cinert cvel), a body per lane; (C) subtree sums of the forces — limb
  // suffix sums per lane, a team sum at the trunk, the root path on every lane.
  static constexpr int RCA = TL::RCA, RFB = TL::RFB;  // body accelerations / body forces (scratch)

  // cvel/cacc of the free-joint root body (every lane); its cdof_dot rows go to CDD1 (sensors)
  static DK void root_motion(LP L, int lane, int b, float* cv, float* ca) {
    const int da = Md::body_dofadr[b], nd = Md::body_dofnum[b];
    if (nd == 6) {
      // free joint: the translational cdof rows are the unit vectors e_3..e_5 (com_pos)
      for (int i = 0; i < 3; i++) cv[3 + i] += L[Ly::QVEL + da + i];
      float cvt[6];
      for (int k = 0; k < 6; k++) cvt[k] = cv[k];
      for (int i = 3; i < 6; i++) {
        float cd[6], cdd[6];
        for (int k = 0; k < 6; k++) cd[k] = L[Ly::CDOF + 6 * (da + i) + k];
        cross_motion(cdd, cvt, cd);
        if (lane == i - 3)
          for (int k = 0; k < 6; k++) L[Ly::CDD1 + 6 * (i - 3) + k] = cdd[k];
        const float v = L[Ly::QVEL + da + i];
        for (int k = 0; k < 6; k++) { ca[k] += cdd[k] * v; cv[k] += cd[k] * v; }
      }
    } else {
      for (int jj = 0; jj < nd; jj++) {
        float cd[6], cdd[6];
        for (int k = 0; k < 6; k++) cd[k] = L[Ly::CDOF + 6 * (da + jj) + k];
        cross_motion(cdd, cv, cd);
        const float v = L[Ly::QVEL + da + jj];
        for (int k = 0; k < 6; k++) { ca[k] += cdd[k] * v; cv[k] += cd[k] * v; }
      }
    }
  }

  // PART 0: the whole pass (throughput mode). Latency mode: wave 0 runs rne_vel, then rne_rest<1>
  // (the composite-inertia lanes of phase C write a dump region), wave 1 runs subtree_sums<2> (the
  // composite inertias only: they need com_pos, not the velocities), so crb starts before rne ends
  static DK void rne(LP L, int lane) {
    rne_vel(L, lane);
    rne_rest<0>(L, lane);
  }
  // (A) velocities and accelerations
  static DK void rne_vel(LP L, int lane) {
#pragma clang fp reassociate(on)
    STAGE_T0();
    constexpr int NR = Md::T_NROOT, BL = Md::T_BRLEN, MD = Md::T_BRMD;  // dofs per limb body (2: backlash)
    static_assert(Md::T_NBR <= TEAM, "a limb per lane");
    float cv[6], ca[6];
    for (int k = 0; k < 6; k++) { cv[k] = 0.0f; ca[k] = (k >= 3) ? -Md::gravity[k - 3] : 0.0f; }
#pragma unroll
    for (int r = 0; r < NR; r++) {
      const int b = Md::T_ROOT[r];
      root_motion(L, lane, b, cv, ca);
      if (lane == 0)
        for (int k = 0; k < 6; k++) { L[Ly::CVEL + 6 * b + k] = cv[k]; L[RCA + 6 * b + k] = ca[k]; }
    }
    const bool limb = lane < Md::T_NBR;
    int bb[BL];
#pragma unroll
    for (int d = 0; d < BL; d++) bb[d] = limb_body(lane, d);
    {
      float cd[BL][MD][6], qv[BL][MD];
      int dof[BL][MD];
#pragma unroll
      for (int d = 0; d < BL; d++)
#pragma unroll
        for (int jj = 0; jj < MD; jj++) dof[d][jj] = limb_dof(lane, 2 * d + jj);
#pragma unroll
      for (int d = 0; d < BL; d++)
#pragma unroll
        for (int jj = 0; jj < MD; jj++) {
          const int i = dof[d][jj] >= 0 ? dof[d][jj] : 0;
          for (int k = 0; k < 6; k++) cd[d][jj][k] = L[Ly::CDOF + 6 * i + k];
          const float q = L[Ly::QVEL + i];  // unconditional load, then select (no masked load)
          qv[d][jj] = dof[d][jj] >= 0 ? q : 0.0f;
        }
#pragma unroll
      for (int d = 0; d < BL; d++) {
#pragma unroll
        for (int jj = 0; jj < MD; jj++) {
          float cdd[6];
          cross_motion(cdd, cv, cd[d][jj]);
          const float v = qv[d][jj];
          for (int k = 0; k < 6; k++) { ca[k] += cdd[k] * v; cv[k] += cd[d][jj][k] * v; }
        }
        if (limb && bb[d] >= 0)
          for (int k = 0; k < 6; k++) { L[Ly::CVEL + 6 * bb[d] + k] = cv[k]; L[RCA + 6 * bb[d] + k] = ca[k]; }
      }
    }
    TSYNC();
    STAGE_MARK(21);
  }
  template <int PART>
  static DK void rne_rest(LP L, int lane) {
#pragma clang fp reassociate(on)
    STAGE_T0();
    // (B) body forces, a body per lane
    team_for<NB, 1>(lane, [&](int b) {
      if (!moving(b)) return;
      float I[10], v6[6], a6[6], f[6], t1[6], t2[6];
      for (int k = 0; k < 10; k++) I[k] = L[Ly::CIN + 10 * b + k];
      for (int k = 0; k < 6; k++) { v6[k] = L[Ly::CVEL + 6 * b + k]; a6[k] = L[RCA + 6 * b + k]; }
      mul_inert_vec(f, I, a6);
      mul_inert_vec(t1, I, v6);
      cross_force(t2, v6, t1);
      for (int k = 0; k < 6; k++) L[RFB + 6 * b + k] = f[k] + t2[k];
    });
    TSYNC();
    STAGE_MARK(22);
    // (C) subtree sums of the body forces (rne) and of the body inertias (mj_crb's composite
    // inertias, which overwrite CIN: phase B has read the body inertias), a component per lane:
    // lane k < 6 sums force component k, lane 6 + j inertia component j, down every limb from its
    // tip (the limb bodies are compile-time, Md::T_BRB), then the limb totals, then the root path.
    // Each component's additions run in the same order as a limb-per-lane pass.
    subtree_sums<PART>(L, lane);
    team_for<NV>(lane, [&](int i) {
      const int b = dof_body(i);
      float s = 0.0f;
      for (int k = 0; k < 6; k++) s += L[Ly::CDOF + 6 * i + k] * L[TL::CFRC + 6 * b + k];
      L[Ly::FSM + i] = -s;
    });
    TSYNC();
  }
  static constexpr bool bodies_distinct() {
    for (int m = 0; m < Md::T_NBR; m++)
      for (int d = 0; d < Md::T_BRLEN; d++) {
        const int b = Md::T_BRB[m][d];
        if (b < 0) continue;
        for (int m2 = 0; m2 < Md::T_NBR; m2++)
          for (int d2 = 0; d2 < Md::T_BRLEN; d2++)
            if ((m2 != m || d2 != d) && Md::T_BRB[m2][d2] == b) return false;
        for (int r = 0; r < Md::T_NROOT; r++)
          if (Md::T_ROOT[r] == b) return false;
      }
    for (int r = 0; r < Md::T_NROOT; r++)
      for (int r2 = r + 1; r2 < Md::T_NROOT; r2++)
        if (Md::T_ROOT[r] == Md::T_ROOT[r2]) return false;
    return true;
  }
  // phase C of rne: PART 0 both sums, PART 1 the forces (inertia lanes into XDUM0), PART 2 the
  // composite inertias (force lanes read CIN and write XDUM1: no read of rne's forces in flight)
  template <int PART>
  static DK void subtree_sums(LP L, int lane) {
#pragma clang fp reassociate(on)
    STAGE_T0();
    constexpr int NR = Md::T_NROOT, BL = Md::T_BRLEN;
    static_assert(TEAM == 6 + 10, "a force or inertia component per lane");
    {
      int lk = lane;
      asm volatile("" : "+v"(lk));  // else the per-lane address selects are hoisted out of the substep
                                    // loop into registers (+19 AGPRs, -6 % measured)
      const bool fk = lk < 6;
      const int fsrc = PART == 2 ? Ly::CIN + lk : RFB + lk, fdst = PART == 2 ? TL::XDUM1 + lk : TL::CFRC + lk;
      const int idst = PART == 1 ? TL::XDUM0 + (lk - 6) : TL::XCIN + (lk - 6);
      const int src = fk ? fsrc : Ly::CIN + (lk - 6), dst = fk ? fdst : idst;
      const int st = fk ? 6 : 10;
      // every body's word first, in one batch: the bodies are distinct (bodies_distinct), so no store
      // below (in place for the inertias in throughput mode) feeds a later read. Interleaved, the
      // loads could not pass the stores (same region) and each body cost an LDS round trip
      static_assert(bodies_distinct(), "limb and root bodies must be distinct");
      float xb[Md::T_NBR][BL], xr[NR];
#pragma unroll
      for (int m = 0; m < Md::T_NBR; m++)
#pragma unroll
        for (int d = 0; d < BL; d++) {
          const int b = Md::T_BRB[m][d];
          xb[m][d] = b >= 0 ? L[src + st * (b >= 0 ? b : 0)] : 0.0f;
        }
#pragma unroll
      for (int r = 0; r < NR; r++) xr[r] = L[src + st * Md::T_ROOT[r]];
      float tot = 0.0f;
#pragma unroll
      for (int m = 0; m < Md::T_NBR; m++) {
        float acc = 0.0f;
#pragma unroll
        for (int d = BL - 1; d >= 0; d--) {
          const int b = Md::T_BRB[m][d];
          if (b < 0) continue;
          acc += xb[m][d];
          L[dst + st * b] = acc;
        }
        tot = m == 0 ? acc : tot + acc;
      }
      STAGE_MARK(35);
#pragma unroll
      for (int r = NR - 1; r >= 0; r--) {
        const int b = Md::T_ROOT[r];
        tot += xr[r];
        L[dst + st * b] = tot;
      }
    }
    TSYNC();
    STAGE_MARK(36);
  }

  // ---------------- mj_crb: the sparse M from the composite inertias (summed in rne) ----
  static DK void crb(LP L, int lane) {
#pragma clang fp reassociate(on)
    STAGE_T0();
    constexpr int BL = Md::T_BRLEN, MC = Md::MAXCHAIN;
    // (the composite inertias were summed in rne's subtree pass)
    STAGE_MARK(19);
#ifdef DUCK_ASM_MARKS
    asm volatile("; CRB_BEGIN" ::: "memory");
#endif
    L[lane == 0 ? Ly::MZERO : TL::SINK + lane] = 0.0f;  // the zero word load_cols reads (LDS is not
                                                          // initialised by the launch)
    // M row i (lane i, i + 16): F_i = crb_{body(i)} cdof_i stays in registers;
    // M[i][j] = cdof_j . F_i over the ancestors j of i (the row is contiguous in M)
    // a last column set of at most 4 rows takes 4 lanes per row, each lane a quarter of the row's
    // entries (otherwise 4 lanes do the whole set's work while 12 idle)
    constexpr int RT = NV - TEAM * (NC - 1);
    constexpr bool SPLIT = NC >= 2 && RT <= 4;
    constexpr int NS = SPLIT ? NC - 1 : NC;
#pragma unroll
    for (int s = 0; s < NS; s++) {
      const int i = TEAM * s + lane, ic = i < NV ? i : 0;
      float cd[6], F[6], I[10];
      for (int k = 0; k < 6; k++) cd[k] = L[Ly::CDOF + 6 * ic + k];
      const int bi = dof_body(ic);
      for (int k = 0; k < 10; k++) I[k] = L[TL::XCIN + 10 * bi + k];
      int jj[MC];
      float cj[MC][6];
      // with B_DCHAFF the chain is the B_DCHN free-joint dofs, then the run of limb dofs from the
      // run start at or below i up to i (codegen T_DLST): no index words to load
      int st = Md::T_DLST[0];
#pragma unroll
      for (int k = 1; k < Md::T_NDLST; k++) st = ic >= Md::T_DLST[k] ? Md::T_DLST[k] : st;
#pragma unroll
      for (int q = 0; q < MC; q++) {
        if constexpr (Md::B_DCHAFF) {
          constexpr int NF = Md::B_DCHN;
          const int jq = q < NF ? q : st + (q - NF);
          jj[q] = (q < NF ? (ic < NF ? q <= ic : true) : (ic >= NF && jq <= ic)) ? jq : -1;
        } else {
          jj[q] = ti(Md::B_DCHAIN + MC * ic + q);
        }
        if (FREE0 && q < 3) continue;  // ancestors ascending: position q < 3 is dof q, cdof = e_{3+q}
        const int jc = jj[q] >= 0 ? jj[q] : 0;
        for (int k = 0; k < 6; k++) cj[q][k] = L[Ly::CDOF + 6 * jc + k];
      }
      const float arm = L[Ly::DARM + ic];
      const int rs = ti(Md::B_MROW + ic);
      mul_inert_vec(F, I, cd);
#pragma unroll
      for (int q = 0; q < MC; q++) {
        float v = 0.0f;
        if (FREE0 && q < 3)
          v = F[3 + q];  // cdof_q = e_{3+q}
        else
          for (int k = 0; k < 6; k++) v += cj[q][k] * F[k];
        // branchless store (a masked region per entry costs more than the select)
        const bool ok = i < NV && jj[q] >= 0;
        L[ok ? Ly::M + rs + q : TL::SINK + lane] = v + (jj[q] == i ? arm : 0.0f);
      }
    }
    if constexpr (SPLIT) {
      int lr = lane;
      asm volatile("" : "+v"(lr));  // the per-lane row/entry split stays inside the substep
      const int i = TEAM * (NC - 1) + (lr >> 2), sub = lr & 3;
      const bool okr = i < NV;
      const int ic = okr ? i : 0;
      float cd[6], F[6], I[10];
      for (int k = 0; k < 6; k++) cd[k] = L[Ly::CDOF + 6 * ic + k];
      const int bi = dof_body(ic);
      for (int k = 0; k < 10; k++) I[k] = L[TL::XCIN + 10 * bi + k];
      const float arm = L[Ly::DARM + ic];
      const int rs = ti(Md::B_MROW + ic);
      mul_inert_vec(F, I, cd);
#pragma unroll
      for (int t = 0; t < (MC + 3) / 4; t++) {
        const int q = sub + 4 * t;
        const bool okq = q < MC;
        const int qc = okq ? q : 0;
        const int j = ti(Md::B_DCHAIN + MC * ic + qc), jc = j >= 0 ? j : 0;
        float cj[6];
        for (int k = 0; k < 6; k++) cj[k] = L[Ly::CDOF + 6 * jc + k];
        float v = 0.0f;
        for (int k = 0; k < 6; k++) v += cj[k] * F[k];
        if (FREE0) v = qc < 3 ? (qc == 0 ? F[3] : (qc == 1 ? F[4] : F[5])) : v;  // cdof_q = e_{3+q}
        const bool ok = okr && okq && j >= 0;
        L[ok ? Ly::M + rs + qc : TL::SINK + lr] = v + (j == i ? arm : 0.0f);
      }
    }
    TSYNC();
  }

  // ---------------- actuation + passive; H = M ----------------
  static DK void smooth(LP L, int lane) {
#ifdef DUCK_ASM_MARKS
    asm volatile("; SMOOTH_BEGIN" ::: "memory");
#endif
    team_for<NV>(lane, [&](int i) { L[Ly::FSM + i] += -tf(Md::B_DAMP + i) * L[Ly::QVEL + i]; });
    TSYNC();
    if (lane < NU) {
      const int a = lane, o = Md::B_ACT + 12 * a;
      const int dof = act_dof(a);
      float c = L[Ly::CTRL + a];
      if (ti(o)) c = fminf(fmaxf(c, tf(o + 1)), tf(o + 2));
      const float g = tf(o + 3), kp = L[Ly::DKP + a];
      const float len = g * L[Ly::QPOS + act_qadr(a)], vel = g * L[Ly::QVEL + dof];
      float f = kp * c + (-kp * len - tf(o + 6) * vel);
      if (ti(o + 7)) f = fminf(fmaxf(f, tf(o + 8)), tf(o + 9));
      L[Ly::AF + a] = f;
      L[Ly::FSM + dof] += g * f;
    }
    TSYNC();
  }

  // ---------------- register-resident LDL' (mj_factorM + mj_solveLD) ----------------
  // Lane l holds column c = 16 s + l of the matrix densely in registers (col[s][row]); a pivot
  // reads H[K][I] from the lane owning column I with a DPP row broadcast (row_newbcast), so
  // a pass is a handful of broadcasts and FMAs with no memory traffic. Entries above the
  // diagonal may collect garbage; factor_solve zeroes them before the triangular solves.
  static constexpr int NC = (NV + TEAM - 1) / TEAM;
  struct Fac {
    float col[NC][NV];
    float dg[NC];
  };
  template <int SRC>
  static DK float bc(float v) { return dppf<0x150 + SRC>(v); }

  // Pivot K: every lane c updates its column at each ancestor row I of K,
  // H[I][c] -= (H[K][I] / H[K][K]) H[K][c], with H[K][I] read from lane I's register by the DPP
  // operand of one v_mul (row_newbcast), then scales its entry H[K][c]. Column sets s whose
  // columns all lie right of row I (TEAM s > I) hold only above-diagonal entries there and are
  // skipped at compile time. The pivot reciprocal is v_rcp_f32 (1 ulp; pivots are never denormal).
  // The multipliers of all ancestors are formed before the first update (they read row K only, which
  // the updates do not write): with each multiply right before its update, the DPP read of the next
  // ancestor followed a VALU write and took an s_nop (57 per flat step kernel; C2 +0.3 %, C5 +0.65 %).
  template <int K, int I>
  static DK void fac_mult(const Fac& F, float inv, float* t) {
    if constexpr (I >= 0) {
      t[I] = bc<I % TEAM>(F.col[I / TEAM][K]) * inv;
      fac_mult<K, Md::dof_parentid[I]>(F, inv, t);
    }
  }
  template <int K, int I>
  static DK void fac_upd(Fac& F, const float* t) {
    if constexpr (I >= 0) {
#pragma unroll
      for (int s = 0; s < NC; s++)
        if (TEAM * s <= I) F.col[s][I] -= t[I] * F.col[s][K];
      fac_upd<K, Md::dof_parentid[I]>(F, t);
    }
  }
  template <int K>
  static DK void fac_pass(Fac& F, int lane) {
    constexpr int ks = K / TEAM, kl = K % TEAM;
    const float dk = bc<kl>(F.col[ks][K]);
    F.dg[ks] = lane == kl ? F.col[ks][K] : F.dg[ks];
    const float inv = __builtin_amdgcn_rcpf(dk);
    float t[NV];
    fac_mult<K, Md::dof_parentid[K]>(F, inv, t);
    fac_upd<K, Md::dof_parentid[K]>(F, t);
    // scale row K of every column; the diagonal entry (lane kl) becomes 1, never read again
    // (D is kept in dg; the solves read only the strictly lower triangle)
#pragma unroll
    for (int s = 0; s < NC; s++)
      if (TEAM * s <= K) F.col[s][K] *= inv;
  }
  template <int K>
  static DK void sol_back(const Fac& F, float* x) {
    const float xk = bc<K % TEAM>(x[K / TEAM]);
#pragma unroll
    for (int s = 0; s < NC; s++)
      if (TEAM * s < K) x[s] -= F.col[s][K] * xk;
  }
  // lanes holding the ancestors of dof K (bit l: some column c = TEAM s + l is an ancestor of K): the
  // only nonzeros of row K of the tree-sparse factor (the dense factor uses sol_fwd_dense)
  static constexpr unsigned anc_lanes(int K) {
    unsigned m = 0;
    for (int j = Md::dof_parentid[K]; j >= 0; j = Md::dof_parentid[j]) m |= 1u << (j % TEAM);
    return m;
  }
  // sum of v over the lanes in `lanes`, delivered (at least) to lane `dst`: one row broadcast for a
  // single lane, a quad (2 steps) or 8-lane half (3 steps) when lanes and dst share it, else the team sum
  template <unsigned LANES, int DST>
  static DK float anc_sum(float v) {
    constexpr unsigned all = LANES | (1u << DST);
    if constexpr (LANES == 0) {
      return 0.0f;
    } else if constexpr ((LANES & (LANES - 1)) == 0) {
      return bc<__builtin_ctz(LANES)>(v);
    } else if constexpr ((all & ~(0xFu << (4 * (DST / 4)))) == 0) {
      v += dppf<0xB1>(v);  // quad_perm [1,0,3,2]
      v += dppf<0x4E>(v);  // quad_perm [2,3,0,1]
      return v;
    } else if constexpr ((all & ~(0xFFu << (8 * (DST / 8)))) == 0) {
      return hsum8(v);
    } else {
      return tsum(v);
    }
  }
  template <int K>
  static DK void sol_fwd(const Fac& F, float* x, int lane) {
    constexpr unsigned A = anc_lanes(K);
    if constexpr (A != 0) {
      float p = 0.0f;
#pragma unroll
      for (int s = 0; s < NC; s++)
        if (TEAM * s < K) p += F.col[s][K] * x[s];
      p = anc_sum<A, K % TEAM>(p);
      if (lane == K % TEAM) x[K / TEAM] -= p;
    }
  }
  template <int... J>
  static DK void fac_all(Fac& F, int lane, std::integer_sequence<int, J...>) {
    (fac_pass<Md::T_PORD[J]>(F, lane), ...);  // leaves first, limbs interleaved (codegen.pivot_order)
  }
  template <int... J>
  static DK void back_all(const Fac& F, float* x, std::integer_sequence<int, J...>) {
    (sol_back<Md::T_PORD[J]>(F, x), ...);
  }
  template <int... J>
  static DK void fwd_all(const Fac& F, float* x, int lane, std::integer_sequence<int, J...>) {
    (sol_fwd<Md::T_PORD[NV - 1 - J]>(F, x, lane), ...);
  }

  // factor F.col (tree-sparse SPD matrix; only the lower triangle is read, entries right of
  // the diagonal may hold anything) in place and
  // solve for x (lane l holds x[l], x[l+16])
  static DK void factor_solve(Fac& F, float* x, int lane) {
    factor(F, lane);
    solve_factored(F, x, lane);
  }
  static DK void factor(Fac& F, int lane) {
#pragma unroll
    for (int s = 0; s < NC; s++) F.dg[s] = 1.0f;
    fac_all(F, lane, std::make_integer_sequence<int, NV>{});
    // keep the strictly lower triangle (the unit diagonal and the upper garbage become 0): the
    // tree-sparse factor has no fill-in outside ancestor pairs, so the solves need no masks
#pragma unroll
    for (int s = 0; s < NC; s++)
#pragma unroll
      for (int r = TEAM * s + 1; r < NV; r++) F.col[s][r] = lane < r - TEAM * s ? F.col[s][r] : 0.0f;
  }
  static DK void solve_factored(const Fac& F, float* x, int lane) {
    back_all(F, x, std::make_integer_sequence<int, NV>{});
#pragma unroll
    for (int s = 0; s < NC; s++) x[s] = x[s] * __builtin_amdgcn_rcpf(F.dg[s]);
    fwd_all(F, x, lane, std::make_integer_sequence<int, NV>{});
  }
  // out of line so the rare dense path does not share the hot path's code layout / registers
  static DNI void newton_dense(LP L, int lane) {
    float Mc[NC][NV];
    load_cols(L, lane, Mc, false);
    newton_fused<true>(L, lane, Mc);
  }
  // dense variant (a full lower triangle): pivots in natural order NV-1 .. 0, each updating every
  // row above it; then the same mask-free solves, also in natural order
  template <int K, int I>
  static DK void fac_rows_dense(Fac& F, float inv) {
    if constexpr (I >= 0) {
      const float t = bc<I % TEAM>(F.col[I / TEAM][K]) * inv;
#pragma unroll
      for (int s = 0; s < NC; s++)
        if (TEAM * s <= I) F.col[s][I] -= t * F.col[s][K];
      fac_rows_dense<K, I - 1>(F, inv);
    }
  }
  template <int K>
  static DK void fac_pass_dense(Fac& F, int lane) {
    constexpr int ks = K / TEAM, kl = K % TEAM;
    const float dk = bc<kl>(F.col[ks][K]);
    F.dg[ks] = lane == kl ? F.col[ks][K] : F.dg[ks];
    const float inv = __builtin_amdgcn_rcpf(dk);
    fac_rows_dense<K, K - 1>(F, inv);
#pragma unroll
    for (int s = 0; s < NC; s++)
      if (TEAM * s <= K) F.col[s][K] *= inv;
  }
  template <int... J>
  static DK void fac_all_dense(Fac& F, int lane, std::integer_sequence<int, J...>) {
    (fac_pass_dense<NV - 1 - J>(F, lane), ...);
  }
  template <int... J>
  static DK void back_all_dense(const Fac& F, float* x, std::integer_sequence<int, J...>) {
    (sol_back<NV - 1 - J>(F, x), ...);
  }
  // the dense factor has a full lower triangle: every row's dot product needs the whole team sum
  template <int K>
  static DK void sol_fwd_dense(const Fac& F, float* x, int lane) {
    float p = 0.0f;
#pragma unroll
    for (int s = 0; s < NC; s++)
      if (TEAM * s < K) p += F.col[s][K] * x[s];
    p = tsum(p);
    if (lane == K % TEAM) x[K / TEAM] -= p;
  }
  template <int... J>
  static DK void fwd_all_dense(const Fac& F, float* x, int lane, std::integer_sequence<int, J...>) {
    (sol_fwd_dense<J>(F, x, lane), ...);
  }
  static DK void factor_solve_dense(Fac& F, float* x, int lane) {
#pragma unroll
    for (int s = 0; s < NC; s++) F.dg[s] = 1.0f;
    fac_all_dense(F, lane, std::make_integer_sequence<int, NV>{});
#pragma unroll
    for (int s = 0; s < NC; s++)
#pragma unroll
      for (int r = TEAM * s + 1; r < NV; r++) F.col[s][r] = lane < r - TEAM * s ? F.col[s][r] : 0.0f;
    back_all_dense(F, x, std::make_integer_sequence<int, NV>{});
#pragma unroll
    for (int s = 0; s < NC; s++) x[s] = x[s] * __builtin_amdgcn_rcpf(F.dg[s]);
    fwd_all_dense(F, x, lane, std::make_integer_sequence<int, NV>{});
  }

  // columns of the symmetric tree-sparse M: full (both triangles) or lower only. Entries outside
  // the tree pattern (and columns past NV) read the zero word after M: one load per entry, no mask
  static DK void load_cols(LP L, int lane, float (*col)[NV], bool lower_only) {
    if constexpr (TL::TAB_LDS) {
      // lane opaque: the table words are per-lane constants, which the compiler would otherwise
      // hoist out of the substep loop and keep in registers (+39 AGPRs)
      asm volatile("" : "+v"(lane));
      // in groups of G entries: G table words, then G M words. Written entry by entry, the
      // scheduler (short of registers here) alternated one table load and one M load with a wait
      // for each: 2 NV dependent LDS round trips per substep (C5 +2.3 %; with a scheduling barrier
      // between the groups C2 lost 0.9 %, without one it gains 0.6 %)
      constexpr int G = 10;
#pragma unroll
      for (int s = 0; s < NC; s++) {
#pragma unroll
        for (int r0 = 0; r0 < NV; r0 += G) {
          int a[G];
#pragma unroll
          for (int r = r0; r < r0 + G && r < NV; r++)
            if (!(lower_only && r < TEAM * s)) a[r - r0] = ti(Md::B_MCOLZ + TEAM * (NV * s + r) + lane);
#pragma unroll
          for (int r = r0; r < r0 + G && r < NV; r++) {
            if (lower_only && r < TEAM * s) { col[s][r] = 0.0f; continue; }  // above the diagonal
            // (with lower_only the entries right of the diagonal may stay: the factorization's lower
            // triangle never reads them, and factor_solve drops them afterwards)
            col[s][r] = L[Ly::M + a[r - r0]];
          }
        }
      }
    } else {
      // model tables in global memory (models whose env slices leave no LDS for them): the M
      // addresses of the pattern are loop-invariant index words the compiler keeps in registers
      // across the substeps, so the masked form without the per-launch table reads is faster
#pragma unroll
      for (int s = 0; s < NC; s++) {
        const int c = TEAM * s + lane, cc = c < NV ? c : 0;
#pragma unroll
        for (int r = 0; r < NV; r++) {
          const int a = madr(r, cc);
          if (lower_only && r < TEAM * s) { col[s][r] = 0.0f; continue; }
          const float v = L[Ly::M + (a >= 0 ? a : 0)];  // unconditional load: no branch per entry
          col[s][r] = (c < NV && a >= 0) ? v : 0.0f;
        }
      }
    }
  }

  // qacc_smooth = M^-1 qfrc_smooth (mj_solveM) from the solver's register columns of M: the factor
  // works on a copy (it reads only the lower triangle) and Mc stays for every M.x of the solver,
  // so M is loaded from LDS once per substep
  static DK void smooth_acc(LP L, int lane, const float (*Mc)[NV]) {
    Fac F;
#pragma unroll
    for (int s = 0; s < NC; s++)
#pragma unroll
      for (int r = 0; r < NV; r++) F.col[s][r] = Mc[s][r];
    float x[NC];
#pragma unroll
    for (int s = 0; s < NC; s++) {
      const int c = TEAM * s + lane;
      const float v = L[Ly::FSM + (c < NV ? c : 0)];
      x[s] = c < NV ? v : 0.0f;
    }
    factor_solve(F, x, lane);
#pragma unroll
    for (int s = 0; s < NC; s++) {
      const int c = TEAM * s + lane;
      if (c < NV) L[Ly::QSM + c] = x[s];
    }
    TSYNC();
  }
  // (latency mode: the factorization runs before qfrc_smooth is known, the solve after)
  static DK void smooth_factor(Fac& F, int lane, const float (*Mc)[NV]) {
#pragma unroll
    for (int s = 0; s < NC; s++)
#pragma unroll
      for (int r = 0; r < NV; r++) F.col[s][r] = Mc[s][r];
    factor(F, lane);
  }
  static DK void smooth_solve(LP L, int lane, const Fac& F) {
    float x[NC];
#pragma unroll
    for (int s = 0; s < NC; s++) {
      const int c = TEAM * s + lane;
      const float v = L[Ly::FSM + (c < NV ? c : 0)];
      x[s] = c < NV ? v : 0.0f;
    }
    solve_factored(F, x, lane);
#pragma unroll
    for (int s = 0; s < NC; s++) {
      const int c = TEAM * s + lane;
      if (c < NV) L[Ly::QSM + c] = x[s];
    }
    TSYNC();
  }

  // y = M x for the lane's columns (M held as full columns); Y[c] = y. x[s] holds x_c of the lane's
  // columns c = TEAM s + lane; x_r reaches every lane by a DPP row broadcast folded into the FMA
  template <int... R>
  static DK void mul_acc(const float (*Mc)[NV], const float* x, float* y, std::integer_sequence<int, R...>) {
#pragma unroll
    for (int s = 0; s < NC; s++) ((y[s] += Mc[s][R] * bc<R % TEAM>(x[R / TEAM])), ...);
  }
  static DK void mul_cols(LP L, int lane, const float (*Mc)[NV], const float* x, int Y) {
    float y[NC];
#pragma unroll
    for (int s = 0; s < NC; s++) y[s] = 0.0f;
    mul_acc(Mc, x, y, std::make_integer_sequence<int, NV>{});
#pragma unroll
    for (int s = 0; s < NC; s++) {
      const int c = TEAM * s + lane;
      if (c < NV) L[Y + c] = y[s];
    }
  }
  // the lane's entries x[s] = X[TEAM s + lane] of an LDS vector
  static DK void lane_vec(LP L, int lane, int X, float* x) {
#pragma unroll
    for (int s = 0; s < NC; s++) {
      const int c = TEAM * s + lane;
      x[s] = L[X + (c < NV ? c : 0)];
    }
  }

  static constexpr unsigned chain_mask(int b) {
    unsigned msk = 0;
    for (int q = 0; q < Md::chain_len[b]; q++) msk |= 1u << Md::chain[b][q];
    return msk;
  }

  // H[r][c] += kc_r . cdof_c for the chain rows r on or below the diagonal block of each column set
  // (kc_r read from lane r % TEAM of set r / TEAM); kc_r = 0 off the chain
  template <int R>
  static DK void jdj_row(Fac& F, const float (*kc)[6], const float (*cdc)[6], const bool* in, unsigned msk) {
    if (!((msk >> R) & 1u)) return;  // compile-time after unrolling (msk is the side's constant)
#pragma unroll
    for (int s = 0; s < NC; s++) {
      if (R < TEAM * s) continue;
      if (FREE0 && R < 3) { F.col[s][R] += kc[s][3 + R]; continue; }  // cdof_r = e_{3+r}
      float h = 0.0f;
      for (int k = 0; k < 6; k++) h += bc<R % TEAM>(kc[R / TEAM][k]) * cdc[s][k];
      F.col[s][R] += in[s] ? h : 0.0f;  // (entries right of the diagonal are dropped after the factorization)
    }
  }
  template <int... R>
  static DK void jdj_rows(Fac& F, const float (*kc)[6], const float (*cdc)[6], const bool* in, unsigned msk,
                          std::integer_sequence<int, R...>) {
    (jdj_row<R>(F, kc, cdc, in, msk), ...);
  }

  // Newton direction at (QACC, JA, MA) with H = M + J'DJ assembled directly into register
  // columns (mjx _update_gradient + the Cholesky solve): SRCH = -H^-1 grad. Returns false
  // (nothing written) when foot/foot contact rows are active.
  // FF = false: the common case, tree-sparse H (returns false, nothing written, when foot/foot
  // contact rows are active). FF = true: those rows included — their Jacobian J_geom2 - J_geom1
  // couples the two legs, so H is assembled densely and factored by factor_solve_dense.
  template <bool FF, int OUT = Ly::SRCH>
  static DK bool newton_fused(LP L, int lane, const float (*Mc)[NV]) {
    STAGE_T0();
    if constexpr (!FF) {
      if (Md::FOOT_PAIR >= 0) {
        const int row = R_CON + 16 * Md::FOOT_PAIR + lane;
        const float act = (L[Ly::JA + row] < 0.0f && L[Ly::RD + row] != 0.0f) ? 1.0f : 0.0f;
        if (tsum(act) > 0.0f) return false;
      }
    }
    Fac F;
    float g[NC];
#pragma unroll
    for (int s = 0; s < NC; s++) {
      const int c = TEAM * s + lane, cc = c < NV ? c : 0;
      const bool valid = c < NV;
      float gr = L[Ly::MA + cc] - L[Ly::FSM + cc], diag = 0.0f;
      // friction row of dof c (Huber cost): force and quadratic-zone curvature
      const int fr = dof_fric(cc), frc = fr >= 0 ? fr : 0;
      {
        const float D = L[Ly::RD + frc], x = L[Ly::JA + frc], f = L[Ly::DFRIC + cc], rf = f * frcp(D);
        const float force = x <= -rf ? f : (x >= rf ? -f : -D * x);
        const bool quad = x > -rf && x < rf;
        gr -= fr >= 0 ? force : 0.0f;
        diag += (fr >= 0 && quad) ? D : 0.0f;
      }
      // joint-limit row of dof c (one-sided)
      const int lr = dof_lim(cc), lrc = lr >= 0 ? lr : 0;
      {
        const float D = L[Ly::RD + R_LIM + lrc], x = L[Ly::JA + R_LIM + lrc], sg = L[Ly::LSGN + lrc];
        const bool act = lr >= 0 && x < 0.0f;
        gr -= act ? sg * (-D * x) : 0.0f;
        diag += act ? D : 0.0f;
      }
      g[s] = valid ? gr : 0.0f;
#pragma unroll
      for (int r = 0; r < NV; r++) F.col[s][r] = r >= TEAM * s ? Mc[s][r] + (r == c ? diag : 0.0f) : 0.0f;
    }
    STAGE_MARK(16);
    // contact rows of each floor pair: per-foot 6x6 J'DJ block and J'force. Lanes 0-7 take the
    // 16 rows of side 0's pair, lanes 8-15 side 1's (two rows per lane), each half sums its
    // 27 values over 8 lanes; each side's sums are then broadcast from lane 0 or 8
    float Kh[21], Fh[6];
    {
      const int hs = lane >> 3, l8 = lane & 7;
      const int p = hs == 0 ? Md::PLANE_PAIR[0] : Md::PLANE_PAIR[1];
      const float mu = tf(Md::B_PAIR + PAIRW * p + 2);
#pragma unroll
      for (int k = 0; k < 21; k++) Kh[k] = 0.0f;
#pragma unroll
      for (int k = 0; k < 6; k++) Fh[k] = 0.0f;
#pragma unroll
      for (int h2 = 0; h2 < 2; h2++) {
        const int j = l8 + 8 * h2, slot = 4 * p + (j >> 2), e = j & 3, row = R_CON + 4 * slot + e;
        const float D = L[Ly::RD + row], x = L[Ly::JA + row];
        const float w = (x < 0.0f && D != 0.0f) ? D : 0.0f;
        const float force = -w * x;
        const int t = 1 + (e >> 1);
        const float sg = (e & 1) ? -mu : mu;
        float u[3], r3[3], a[6];
        for (int q = 0; q < 3; q++) {
          u[q] = L[Ly::CFR + 9 * slot + q] + sg * L[Ly::CFR + 9 * slot + 3 * t + q];
          r3[q] = L[Ly::CR + 3 * slot + q];
        }
        cross3(a, r3, u);
        a[3] = u[0]; a[4] = u[1]; a[5] = u[2];
        int o = 0;
        for (int q = 0; q < 6; q++)
          for (int kk = q; kk < 6; kk++) { Kh[o] += w * a[q] * a[kk]; o++; }
        for (int q = 0; q < 6; q++) Fh[q] += force * a[q];
      }
#pragma unroll
      for (int k = 0; k < 21; k++) Kh[k] = hsum8(Kh[k]);
#pragma unroll
      for (int k = 0; k < 6; k++) Fh[k] = hsum8(Fh[k]);
    }
#pragma unroll
    for (int side = 0; side < 2; side++) {
      const int p = Md::PLANE_PAIR[side];
      const int foot = cgeom_slot<Md>(Md::pair_geom2[p]);  // 1 left, 2 right
      float K[21], Fv[6];
#pragma unroll
      for (int k = 0; k < 21; k++) K[k] = side == 0 ? bc<0>(Kh[k]) : bc<8>(Kh[k]);
#pragma unroll
      for (int k = 0; k < 6; k++) Fv[k] = side == 0 ? bc<0>(Fh[k]) : bc<8>(Fh[k]);
      constexpr unsigned MASKL = chain_mask(Md::LFOOT_BODY), MASKR = chain_mask(Md::RFOOT_BODY);
      const unsigned msk = foot == 1 ? MASKL : MASKR;
      // kc_c = K cdof_c for both column sets first: H[r][c] += cdof_r . K cdof_c = kc_r . cdof_c
      // (K symmetric) takes kc_r from lane r by a DPP row broadcast folded into the FMA, instead of
      // reloading cdof_r from LDS in every lane
      float cdc[NC][6], kc[NC][6];
      bool in[NC];
#pragma unroll
      for (int s = 0; s < NC; s++) {
        const int c = TEAM * s + lane, cc = c < NV ? c : 0;
        in[s] = c < NV && ((msk >> cc) & 1u);
        for (int k = 0; k < 6; k++) cdc[s][k] = L[Ly::CDOF + 6 * cc + k];
        float gf = 0.0f;
        for (int q = 0; q < 6; q++) {
          float sacc = 0.0f;
          for (int k = 0; k < 6; k++) sacc += K[kidx(q, k)] * cdc[s][k];
          kc[s][q] = in[s] ? sacc : 0.0f;
          gf += cdc[s][q] * Fv[q];
        }
        g[s] -= in[s] ? gf : 0.0f;
      }
      jdj_rows(F, kc, cdc, in, msk, std::make_integer_sequence<int, NV>{});
    }
    if constexpr (FF) {
      if constexpr (Md::FOOT_PAIR >= 0) {
        // foot/foot rows: J = a . (S_2 - S_1) with S_k the cdof columns of geom k's body chain
        // (shared free-joint dofs cancel); K_ff, F_ff by team sums, then signed projections
        constexpr int p = Md::FOOT_PAIR;
        constexpr int g1 = cgeom_slot<Md>(Md::pair_geom1[p]), g2 = cgeom_slot<Md>(Md::pair_geom2[p]);
        constexpr unsigned M1 = chain_mask(g1 == 1 ? Md::LFOOT_BODY : Md::RFOOT_BODY);
        constexpr unsigned M2 = chain_mask(g2 == 1 ? Md::LFOOT_BODY : Md::RFOOT_BODY);
        const float mu = tf(Md::B_PAIR + PAIRW * p + 2);
        const int slot = 4 * p + (lane >> 2), e = lane & 3, row = R_CON + 4 * slot + e;
        const float D = L[Ly::RD + row], x = L[Ly::JA + row];
        const float w = (x < 0.0f && D != 0.0f) ? D : 0.0f;
        const float force = -w * x;
        const int t = 1 + (e >> 1);
        const float sg = (e & 1) ? -mu : mu;
        float u[3], r3[3], a[6];
        for (int q = 0; q < 3; q++) {
          u[q] = L[Ly::CFR + 9 * slot + q] + sg * L[Ly::CFR + 9 * slot + 3 * t + q];
          r3[q] = L[Ly::CR + 3 * slot + q];
        }
        cross3(a, r3, u);
        a[3] = u[0]; a[4] = u[1]; a[5] = u[2];
        float K[21], Fv[6];
        {
          int o = 0;
          for (int q = 0; q < 6; q++)
            for (int kk = q; kk < 6; kk++) { K[o] = tsum(w * a[q] * a[kk]); o++; }
          for (int q = 0; q < 6; q++) Fv[q] = tsum(force * a[q]);
        }
#pragma unroll
        for (int s = 0; s < NC; s++) {
          const int c = TEAM * s + lane, cc = c < NV ? c : 0;
          const float sc = c < NV ? (float)((int)((M2 >> cc) & 1u) - (int)((M1 >> cc) & 1u)) : 0.0f;
          float cdc[6], kc[6];
          for (int k = 0; k < 6; k++) cdc[k] = sc * L[Ly::CDOF + 6 * cc + k];
          float gf = 0.0f;
          for (int q = 0; q < 6; q++) {
            float sacc = 0.0f;
            for (int k = 0; k < 6; k++) sacc += K[kidx(q, k)] * cdc[k];
            kc[q] = sacc;
            gf += cdc[q] * Fv[q];
          }
          g[s] -= gf;
#pragma unroll
          for (int r = 0; r < NV; r++) {
            const int sr = (int)((M2 >> r) & 1u) - (int)((M1 >> r) & 1u);
            if (sr == 0 || r < TEAM * s) continue;  // compile-time after unrolling
            float h = 0.0f;
            for (int k = 0; k < 6; k++) h += L[Ly::CDOF + 6 * r + k] * kc[k];
            F.col[s][r] += sr > 0 ? h : -h;
          }
        }
      }
    }
    STAGE_MARK(17);
    if constexpr (FF) factor_solve_dense(F, g, lane);
    else factor_solve(F, g, lane);
    STAGE_MARK(18);
#pragma unroll
    for (int s = 0; s < NC; s++) {
      const int c = TEAM * s + lane;
      if (c < NV) L[OUT + c] = -g[s];
    }
    TSYNC();
    return true;
  }

  // ---------------- collision ----------------
  // world frame of collision geom slot gs (1 left foot, 2 right foot: moving bodies)
  static DK void cgeom_frame(LP L, int gs, float* gp, float* gR) {
    const int o = Md::B_CGEOM + 16 * gs, b = ti(o);
    float R[9], t[3], gpos[3], gm[9];
    for (int k = 0; k < 9; k++) { R[k] = L[Ly::XMAT + 9 * b + k]; gm[k] = tf(o + 4 + k); }
    for (int k = 0; k < 3; k++) gpos[k] = tf(o + 1 + k);
    mulmv3(t, R, gpos);
    for (int k = 0; k < 3; k++) gp[k] = L[Ly::XPOS + 3 * b + k] + t[k];
    mulmm3(gR, R, gm);
  }

  // plane floor vs hull for both feet at once (mjx collision_convex.plane_convex): lanes 0-7 take
  // the first floor pair, 8-15 the second
  static DK void collide_planes(LP L, int lane) {
    constexpr int NH = Md::NHV;
    const int h = lane >> 3, sub = lane & 7;
    const int p = Md::PLANE_PAIR[0] * (1 - h) + Md::PLANE_PAIR[1] * h;
    const int gs = cgeom_slot<Md>(Md::pair_geom2[p]);
    float pp[3], PR[9], cp[3], CR[9];
    S1 Ls{L};
    P1::geom_frame(Ls, 0, pp, PR);
    cgeom_frame(L, gs, cp, CR);
    const float n[3] = {PR[2], PR[5], PR[8]};
    const float dif[3] = {pp[0] - cp[0], pp[1] - cp[1], pp[2] - cp[2]};
    float pl[3], nl[3];
    mulmtv3(pl, CR, dif);
    mulmtv3(nl, CR, n);
    auto HVf = [&](int k, int q) { return tf(Md::B_HULL + 3 * k + q); };
    // this lane's vertices: k = sub + 8r
    constexpr int R = (NH + 7) / 8;
    float sup[R], vx[R], vy[R], vz[R];
    float smax = -1e30f;
    for (int r = 0; r < R; r++) {
      const int k = sub + 8 * r;
      const bool ok = k < NH;
      vx[r] = ok ? HVf(k, 0) : 0.0f; vy[r] = ok ? HVf(k, 1) : 0.0f; vz[r] = ok ? HVf(k, 2) : 0.0f;
      sup[r] = ok ? (pl[0] - vx[r]) * nl[0] + (pl[1] - vy[r]) * nl[1] + (pl[2] - vz[r]) * nl[2] : -1e30f;
      smax = fmaxf(smax, sup[r]);
    }
    smax = hmax8(smax);
    const float thr = fmaxf(smax - 1e-3f, 0.0f);
    float dm[R];
    for (int r = 0; r < R; r++) dm[r] = (sub + 8 * r < NH) ? (sup[r] > thr ? 0.0f : -1e6f) : -1e30f;
    // manifold_points (mjx collision_convex._manifold_points), argmax = first index within tol
    auto argmax = [&](const float* v, float tol) -> int {
      float mx = -1e30f;
      for (int r = 0; r < R; r++) mx = fmaxf(mx, v[r]);
      mx = hmax8(mx);
      int best = 1 << 20;
      for (int r = 0; r < R; r++) {
        const int k = sub + 8 * r;
        if (k < NH && v[r] >= mx - tol) best = min(best, k);
      }
      best = hmin8i(best);
      return best < NH ? best : NH - 1;  // argmax_tol's default (also for NaN data)
    };
    auto vert = [&](int k, float* o) { o[0] = HVf(k, 0); o[1] = HVf(k, 1); o[2] = HVf(k, 2); };
    float s[R];
    const int a = argmax(dm, 0.0f);
    float pa[3];
    vert(a, pa);
    for (int r = 0; r < R; r++) {
      const float dx = pa[0] - vx[r], dy = pa[1] - vy[r], dz = pa[2] - vz[r];
      s[r] = dx * dx + dy * dy + dz * dz + dm[r];
    }
    const int b = argmax(s, MANIFOLD_TOL);
    float pb[3];
    vert(b, pb);
    float amb[3] = {pa[0] - pb[0], pa[1] - pb[1], pa[2] - pb[2]}, ab[3];
    cross3(ab, nl, amb);
    for (int r = 0; r < R; r++) {
      const float ap[3] = {pa[0] - vx[r], pa[1] - vy[r], pa[2] - vz[r]};
      s[r] = fabsf(dot3(ap, ab)) + dm[r];
    }
    const int c = argmax(s, MANIFOLD_TOL);
    float pc[3];
    vert(c, pc);
    float amc[3] = {pa[0] - pc[0], pa[1] - pc[1], pa[2] - pc[2]};
    float bmc[3] = {pb[0] - pc[0], pb[1] - pc[1], pb[2] - pc[2]};
    float ac[3], bc[3];
    cross3(ac, nl, amc);
    cross3(bc, nl, bmc);
    // argmax over the 2N array [|bp.bc| + dm ; |ap.ac| + dm]
    int d;
    {
      float s1[R], s2[R];
      float mx = -1e30f;
      for (int r = 0; r < R; r++) {
        const float bp[3] = {pb[0] - vx[r], pb[1] - vy[r], pb[2] - vz[r]};
        const float ap[3] = {pa[0] - vx[r], pa[1] - vy[r], pa[2] - vz[r]};
        s1[r] = fabsf(dot3(bp, bc)) + dm[r];
        s2[r] = fabsf(dot3(ap, ac)) + dm[r];
        mx = fmaxf(mx, fmaxf(s1[r], s2[r]));
      }
      mx = hmax8(mx);
      int best = 1 << 20;
      for (int r = 0; r < R; r++) {
        const int k = sub + 8 * r;
        if (k < NH && s1[r] >= mx - MANIFOLD_TOL) best = min(best, k);
        if (k < NH && s2[r] >= mx - MANIFOLD_TOL) best = min(best, NH + k);
      }
      d = hmin8i(best);
      d = d < 2 * NH ? d : 2 * NH - 1;
      d = d >= NH ? d - NH : d;
    }
    if (sub < 4) {
      const int idx[4] = {a, b, c, d};
      const int me = idx[sub];
      bool unique = true;
      for (int e = 0; e < 4; e++) unique = unique && !(e < sub && idx[e] == me);
      float v[3], vw[3], pos[3], nw[3], fr[9];
      vert(me, v);
      mulmv3(vw, CR, v);
      const float sp = (pl[0] - v[0]) * nl[0] + (pl[1] - v[1]) * nl[1] + (pl[2] - v[2]) * nl[2];
      nw[0] = n[0]; nw[1] = n[1]; nw[2] = n[2];
      for (int q = 0; q < 3; q++) vw[q] += cp[q];
      const float dist = unique ? -sp : 1.0f;
      for (int q = 0; q < 3; q++) pos[q] = vw[q] - 0.5f * dist * nw[q];
      make_frame(fr, nw);
      P1::store_contact(Ls, 4 * p + sub, dist, pos, fr);
    }
  }

  // ---------------- height field: MuJoCo's prism decomposition ----------------
  // oracle/duck_oracle.c collide_hfield_convex in fp32 (MuJoCo mjc_ConvexHField; DESIGN.md §5 item
  // 6): the hull's bounding box in the field's frame selects the sub-grid; each cell's two
  // triangles (MuJoCo's strip triangulation, diagonal (c, r+1)-(c+1, r)) are the tops of prisms
  // down to -size[3]; every prism that passes the height test is collided with the hull by the
  // exact separating-axis penetration over the faces of the Minkowski difference P - H (prism
  // faces, hull faces, edge pairs whose Gauss-map arcs cross; equal overlaps: the first in the
  // oracle's order), one contact per prism at the penetration-weighted centroid of the vertices of
  // each shape inside the other; the 4 slots are filled by mjx's _manifold_points from the
  // deepest. The 8 lanes of a half-team work one prism at a time (hull vertices, faces and edges
  // l + 8j on lane l); prism q's contact is kept by lane q & 7 in its slot q >> 3. The prism's
  // bottom-edge pairs are not tested (the oracle tests them; they are never the minimum while the
  // hull is above the prism's base, 0.1 m under the field: tests/test_oracle_physics.py).
  // Coordinates: "local" = the field's axes with the origin at the hull frame, "mesh" = the hull frame.
  static DK float hmin8f(float v) { return -hmax8_nc(-v); }
  // this lane's rank within its 8-lane half of the wave's ballot word
  static DK unsigned half_bits(unsigned long long b, int lane) {
    const int base = ((int)threadIdx.x & 63) & ~7;
    (void)lane;
    return (unsigned)(b >> base) & 0xFFu;
  }
  // products with the hull's compile-time faces, vertices and edge arcs (literal operands)
  template <int F>
  static DK float nf_dot(const float* x) {
    return cdot<fbits(Md::hull_face_normal[F][0]), fbits(Md::hull_face_normal[F][1]), fbits(Md::hull_face_normal[F][2])>(x);
  }
  template <int K>
  static DK float hv_dot(const float* x) {
    return cdot<fbits(Md::hull_vert[K][0]), fbits(Md::hull_vert[K][1]), fbits(Md::hull_vert[K][2])>(x);
  }
  template <int E>
  static DK float dxc_dot(const float* x) {
    return cdot<fbits(Md::hull_edge_dxc[E][0]), fbits(Md::hull_edge_dxc[E][1]), fbits(Md::hull_edge_dxc[E][2])>(x);
  }
  // the same products for several vectors at once (cdot3v_off / cdot4v / cdot5v / cdot2c)
#define DUCK_C3(A) fbits(A[0]), fbits(A[1]), fbits(A[2])
  template <int F>
  static DK void nf_off_dot3(const float* x, const float* y, const float* z, float* r) {  // offset_F - n_F . (x, y, z)
    cdot3v_off<DUCK_C3(Md::hull_face_normal[F]), fbits(Md::hull_face_offset[F])>(x, y, z, r);
  }
  template <int F>
  static DK void nf_dot4(const float* x, const float* y, const float* z, const float* u, float* r) {
    cdot4v<DUCK_C3(Md::hull_face_normal[F])>(x, y, z, u, r);
  }
  template <int K>
  static DK void hv_dot5(const float* x, const float* y, const float* z, const float* u, const float* w, float* r) {
    cdot5v<DUCK_C3(Md::hull_vert[K])>(x, y, z, u, w, r);
  }
  template <int K>
  static DK void hv_noff5(const float* x, const float* y, const float* z, const float* u, const float* w, const float* o,
                          float* r) {  // o_i - v_K . x_i
    cdot5v_noff<DUCK_C3(Md::hull_vert[K])>(x, y, z, u, w, o, r);
  }
  template <int K>
  static DK void hv_dot2(const float* x, float& ra, float& rb) {  // vertices K and K + 1
    cdot2c<DUCK_C3(Md::hull_vert[K]), DUCK_C3(Md::hull_vert[K + 1])>(x, ra, rb);
  }
  template <int F>
  static DK void nf_dot2(const float* x, float& ra, float& rb) {  // faces F and F + 1
    cdot2c<DUCK_C3(Md::hull_face_normal[F]), DUCK_C3(Md::hull_face_normal[F + 1])>(x, ra, rb);
  }
  template <int E>
  static DK void dxc_dot2(const float* x, float& ra, float& rb) {  // edges E and E + 1
    cdot2c<DUCK_C3(Md::hull_edge_dxc[E]), DUCK_C3(Md::hull_edge_dxc[E + 1])>(x, ra, rb);
  }
#undef DUCK_C3
  template <int F>
  static DK float nf_off_minus(float x) {  // offset_F - x
    float r;
    asm("v_sub_f32_e32 %0, %1, %2" : "=v"(r) : "i"(fbits(Md::hull_face_offset[F])), "v"(x));
    return r;
  }

  // queue and silhouette-list layout of the height-field SAT (collide_hfield / hf_exec), in the
  // env slice: the survivor queue in the H + constraint-row storage (dead until make_rows()),
  // the per-foot silhouette lists in the composite inertias (dead after crb())
  static constexpr int HF_PRIO_T = 5 + Md::NHF, HF_PRIO_V = HF_PRIO_T + 3 * Md::NHE;
  static constexpr int HF_ENT = 28, HF_QH0 = (Ly::H + 3) & ~3;
  static constexpr int HF_QE = (Ly::CR - HF_QH0) / HF_ENT, HF_QR = 4 * HF_QE < 64 ? 4 * HF_QE : 64;
  static constexpr int HF_CINQ = TL::XSIL, HF_SLF = TL::HF_SLF, HF_SLSZ = TL::HF_SLSZ;
  static_assert(Md::FLOOR_TYPE != 1 || HF_QE >= 16, "height-field SAT queue must fit its LDS storage");

  // One prism's separating-axis test against the hull for the lane that runs queue entry E
  // (collide_hfield), in the hull's mesh frame with the hull's compile-time vertices, faces and
  // edges: the screen's minimum over the prism's faces, bottom and the hull's faces is continued
  // with the vertical-edge pairs (the foot's silhouette list) and the top-edge pairs whose Gauss
  // arcs cross (Gregorius' Minkowski-face test over all hull edges, then the overlap of each
  // crossing pair); equal overlaps: the lowest priority (oracle hf_prism_contact's order). Then
  // the contact point (oracle: the penetration-weighted centroid of the vertices of each shape
  // inside the other, or the midpoint of the support features). Writes (depth, normal, point)
  // over the entry's first 8 floats; depth -1 when separated.
#ifdef DUCK_DOUBLE
  // (measurement builds: values the compiler must treat as changed, so that a doubled stage is recomputed)
  template <int N>
  static DK void launder(float* x) {
#pragma unroll
    for (int i = 0; i < N; i++) asm volatile("" : "+v"(x[i]));
  }
#endif
  static DK void hf_exec(lds_float* E, LP L, int tw) {
    STAGE_T0();
    constexpr int NH = Md::NHV, NF = Md::NHF, NE = Md::NHE;
    constexpr int NPW = (3 * NE + 63) / 64;
    static_assert(NPW <= 3, "top-edge pair masks");
    constexpr float DXC = 2.0f * Md::HF_SIZE[0] / (Md::HF_NCOL - 1), DYC = 2.0f * Md::HF_SIZE[1] / (Md::HF_NROW - 1);
    const float GN = 1.0f / sqrtf(DXC * DXC + DYC * DYC);
    const float GX = DYC * GN, GY = DXC * GN;
    lds_f4* E4 = (lds_f4*)E;
    const f4v d0 = E4[0], d1 = E4[1], d2 = E4[2], d3 = E4[3], d4 = E4[4], d5 = E4[5], d6 = E4[6];
    const float Tm[3][3] = {{d0.x, d0.y, d0.z}, {d1.x, d1.y, d1.z}, {d2.x, d2.y, d2.z}};
    const float base = d0.w;
    float mo = d1.w;
    int mp = __float_as_int(d2.w);
    const int tag = __float_as_int(d3.w), tri = tag & 1, foot = tag >> 1;
    const float ntm[3] = {d3.x, d3.y, d3.z}, zc[3] = {d4.x, d4.y, d4.z};
    const float xc[3] = {d5.x, d5.y, d5.z}, yc[3] = {d6.x, d6.y, d6.z};
    // the prism's side normals (triangle kind A: -x, (g_x, g_y), -y; B: -(g_x, g_y), +x, +y)
    float sm[3][3];
    {
      const float sx0 = tri ? -GX : -1.0f, sx1 = tri ? 1.0f : GX;
      const float sy0 = tri ? -GY : 0.0f, sy1 = tri ? 0.0f : GY, sy2 = tri ? 1.0f : -1.0f;
      for (int a = 0; a < 3; a++) {
        sm[0][a] = sx0 * xc[a] + sy0 * yc[a];
        sm[1][a] = sx1 * xc[a] + sy1 * yc[a];
        sm[2][a] = 0.0f * xc[a] + sy2 * yc[a];
      }
    }
    // selects by a runtime index k (pass 2, the winning axis) as v_cndmask on lane masks the
    // compiler cannot see through: written as selects over elements of the Tm / sm arrays they were
    // folded into indexed loads from scratch-memory copies of the arrays, a memory round trip per pair
    auto side = [&](int k, float* o) {  // side normal k
      const unsigned long long m0 = __ballot(k == 0), m1 = __ballot(k == 1);
      for (int a = 0; a < 3; a++) o[a] = vsel(m0, sm[0][a], vsel(m1, sm[1][a], sm[2][a]));
    };
    auto top_edge = [&](int k, float* tm, float* em) {  // top vertex k and the edge to vertex k + 1
      const unsigned long long m0 = __ballot(k == 0), m1 = __ballot(k == 1);
      for (int a = 0; a < 3; a++) {
        tm[a] = vsel(m0, Tm[0][a], vsel(m1, Tm[1][a], Tm[2][a]));
        em[a] = vsel(m0, Tm[1][a], vsel(m1, Tm[2][a], Tm[0][a])) - tm[a];
      }
    };
    // the hull's faces (compile-time normals): the prism's lowest point along n_f, a bottom vertex
    // where n_f leans up the field's z (priority 5 + f; mu is formed after the SAT for these)
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 20
    for (int rep_ = 0; rep_ < 2; rep_++)
#endif
    {
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 20
      float Tm_l[3][3], zc_l[3] = {zc[0], zc[1], zc[2]};
      for (int k = 0; k < 3; k++)
        for (int a = 0; a < 3; a++) Tm_l[k][a] = Tm[k][a];
      launder<9>(&Tm_l[0][0]);
      launder<3>(zc_l);
      const auto& Tm = Tm_l;
      const auto& zc = zc_l;
#endif
      const float hk[3] = {d4.w - base, d5.w - base, d6.w - base};
      static_for<0, NF>([&](auto fI) {
        constexpr int f = fI.value;
        float d[4];
        nf_dot4<f>(zc, Tm[0], Tm[1], Tm[2], d);
        const float nz = fmax_nc(d[0], 0.0f);
        float pf = d[1] - hk[0] * nz;
        pf = fminf(pf, d[2] - hk[1] * nz);
        pf = fminf(pf, d[3] - hk[2] * nz);
        const float ov = nf_off_minus<f>(pf);
        // (equal overlaps keep the lower priority, and mp < 5 + f here: the screen's axes are 0-4 and
        // the faces run in priority order, so the tie test of `take` is always false)
        const bool b = ov < mo;
        mo = b ? ov : mo;
        mp = b ? 5 + f : mp;
      });
    }
    float mu[3] = {0.0f, 0.0f, 0.0f};
    auto take = [&](float ov, int pr, const float* u) {
      const bool b = (ov < mo) | ((ov == mo) & (pr < mp));
      mo = b ? ov : mo;
      mp = b ? pr : mp;
      for (int a = 0; a < 3; a++) mu[a] = b ? u[a] : mu[a];
    };
    // vertical-edge pairs: the prism's support along w is its vertical edge at vertex kk
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 15
    for (int rep_ = 0; rep_ < 2; rep_++)
#endif
    {
      const lds_float* SL = L + ((foot >> 1) - tw) * TL::STRIDE + HF_CINQ + (foot & 1) * HF_SLSZ;
      const lds_int* SLi = (const lds_int*)SL;
      const lds_f4* SLw = (const lds_f4*)(SL + HF_SLF);
      const int n = SLi[0];
      // each entry's words loaded one iteration ahead (the loop waited for its own loads); the load
      // past the list's last entry reads unused words of the slice
      int e_nx = SLi[1];
      f4v w_nx = SLw[0];
      for (int i = 0; i < n; i++) {
        const int e = e_nx;
        const f4v w = w_nx;
        e_nx = SLi[2 + i];
        w_nx = SLw[1 + i];
        const float wv[3] = {w.x, w.y, w.z};
        const float q0 = dot3(wv, Tm[0]), q1 = dot3(wv, Tm[1]), q2 = dot3(wv, Tm[2]);
        const int kk = q0 >= q1 ? (q0 >= q2 ? 0 : 2) : (q1 >= q2 ? 1 : 2);
        take(fmaxf(q0, fmaxf(q1, q2)) - w.w, HF_PRIO_V + 3 * e + kk, wv);
      }
    }
    STAGE_MARK(44);
    // top-edge pairs (hull edge e, prism top edge k: faces ntm, sm_k). Pass 1: the arcs cross when
    // CBA DBA < 0, ADC BDC < 0 and CBA BDC > 0 (C = -n_a, D = -n_b, B x A = sm_k x ntm: CBA =
    // -phi_a), all three products negative: the sign bit of their maximum, bit q = NE k + e of pm.
    // The bits are shifted into 32-bit words in q order (one v_alignbit per pair; placing each bit
    // at its position took a shift, a mask and an or) and bit-reversed into pm afterwards
    unsigned long long pm[3] = {0ull, 0ull, 0ull};
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 12
    for (int rep_ = 0; rep_ < 2; rep_++)
#endif
    {
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 12
      float ntm_l[3] = {ntm[0], ntm[1], ntm[2]}, sm_l[3][3];
      for (int k = 0; k < 3; k++)
        for (int a = 0; a < 3; a++) sm_l[k][a] = sm[k][a];
      launder<3>(ntm_l);
      launder<9>(&sm_l[0][0]);
      const auto& ntm = ntm_l;
      const auto& sm = sm_l;
#endif
      constexpr int NQW = (3 * NE + 31) / 32;
      unsigned qw[NQW];
#pragma unroll
      for (int j = 0; j < NQW; j++) qw[j] = 0u;
      float hx[3][3];
      for (int k = 0; k < 3; k++) cross3(hx[k], sm[k], ntm);
      // (one prism edge at a time: 30 face products live, not 90)
      float ADC[NE];
      // (pairs of products per statement: cdot2c)
      static_for<0, NE / 2>([&](auto eI) { dxc_dot2<2 * eI.value>(ntm, ADC[2 * eI.value], ADC[2 * eI.value + 1]); });
      if constexpr (NE % 2) ADC[NE - 1] = dxc_dot<NE - 1>(ntm);
      // (k a compile-time constant too, so that every pm index is one: a runtime index kept pm in
      // scratch memory, and pass 2's word selects became indexed scratch loads)
      static_for<0, 3>([&](auto kI) {
        constexpr int k = kI.value;
        float phi[NF];
        static_for<0, NF / 2>([&](auto fI) { nf_dot2<2 * fI.value>(hx[k], phi[2 * fI.value], phi[2 * fI.value + 1]); });
        if constexpr (NF % 2) phi[NF - 1] = nf_dot<NF - 1>(hx[k]);
        auto arc = [&](auto eI, float BDC) {
          constexpr int e = decltype(eI)::value, fa = Md::hull_edge_face[e][0], fb = Md::hull_edge_face[e][1];
          const float mx = fmaxf(fmaxf(phi[fa] * phi[fb], ADC[e] * BDC), phi[fa] * BDC);
          constexpr int q = NE * k + e;
          qw[q >> 5] = (qw[q >> 5] << 1) | (__float_as_uint(mx) >> 31);
        };
        static_for<0, NE / 2>([&](auto eI) {
          constexpr int e = 2 * eI.value;
          float b0, b1;
          dxc_dot2<e>(sm[k], b0, b1);
          arc(std::integral_constant<int, e>{}, b0);
          arc(std::integral_constant<int, e + 1>{}, b1);
        });
        if constexpr (NE % 2) arc(std::integral_constant<int, NE - 1>{}, dxc_dot<NE - 1>(sm[k]));
      });
      // word j holds pairs 32 j .. 32 j + n - 1, the first in its top bit
      static_for<0, NQW>([&](auto jI) {
        constexpr int j = jI.value, n = 3 * NE - 32 * j < 32 ? 3 * NE - 32 * j : 32;
        const unsigned r = __builtin_bitreverse32(qw[j]) >> (32 - n);
        pm[j >> 1] |= (unsigned long long)r << (32 * (j & 1));
      });
    }
    STAGE_MARK(45);
#ifdef DUCK_STAGE_PROF
    if (threadIdx.x < 64) {
      // crossing top-edge pairs: all of the wave's survivors (49), hull edges crossing in any of them (50)
      STAGE_ADD(49, (unsigned long long)(__popcll(pm[0]) + __popcll(pm[1]) + __popcll(pm[2])));
      int uni = 0;
      for (int e = 0; e < NE; e++) {
        unsigned long long b3 = 0ull;
        for (int k = 0; k < 3; k++) b3 |= (pm[(NE * k + e) >> 6] >> ((NE * k + e) & 63)) & 1ull;
        uni += __ballot(b3 != 0ull) != 0ull;
      }
      if ((int)threadIdx.x == __ffsll((long long)__ballot(1)) - 1) STAGE_ADD(50, (unsigned long long)uni);
    }
#endif
    // pass 2: each crossing pair's overlap along ev x em
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 11
    const unsigned long long pm_s[3] = {pm[0], pm[1], pm[2]};
    for (int rep_ = 0; rep_ < 2; rep_++) {
      for (int w = 0; w < 3; w++) pm[w] = pm_s[w];
#endif
    while (pm[0] | pm[1] | pm[2]) {
#ifdef DUCK_STAGE_PROF
      if (threadIdx.x < 64 && (int)threadIdx.x == __ffsll((long long)__ballot(1)) - 1) STAGE_ADD(48, 1ull);
#endif
      const bool z0 = pm[0] == 0ull, z1 = pm[1] == 0ull;
      const unsigned long long w = z0 ? (z1 ? pm[2] : pm[1]) : pm[0];
      const int q = (z0 ? (z1 ? 128 : 64) : 0) + __builtin_ctzll(w);
      const unsigned long long wc = w & (w - 1ull);
      pm[0] = z0 ? pm[0] : wc;
      pm[1] = z0 && !z1 ? wc : pm[1];
      pm[2] = z0 && z1 ? wc : pm[2];
      // (the pairs run in q order; the minimum over (overlap, priority p) does not depend on it)
      const int k = q >= 2 * NE ? 2 : (q >= NE ? 1 : 0), e = q - NE * k, p = 3 * e + k, o = Md::B_HEDGE + 20 * e;
      const f4v ev4 = ht4(o + 12), v04 = ht4(o + 16);
      const float ev[3] = {ev4.x, ev4.y, ev4.z}, v0[3] = {v04.x, v04.y, v04.z};
      float em[3], tm[3], sk[3];
      side(k, sk);
      top_edge(k, tm, em);
      float u[3];
      cross3(u, ev, em);
      const float u2 = dot3(u, u);
      const float sg = (dot3(u, ntm) + dot3(u, sk) < 0.0f ? -1.0f : 1.0f) * __builtin_amdgcn_rsqf(u2);
      const float un[3] = {sg * u[0], sg * u[1], sg * u[2]};
      // (a degenerate pair, ev parallel to em, gives no axis; ev4.w = |ev|^2)
      const float ov = u2 >= 1e-12f * ev4.w * dot3(em, em) ? sg * (dot3(u, tm) - dot3(u, v0)) : 1e30f;
      take(ov, HF_PRIO_T + p, un);
    }
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 11
    }
#endif
    STAGE_MARK(47);
    if (!(mo > 0.0f)) {
      E4[0] = f4v{-1.0f, 0.0f, 0.0f, 0.0f};
      return;
    }
    // the screen's axes: the prism's top, sides, bottom or a hull face
    if (mp < HF_PRIO_T) {
      const int f = mp - 5;
      const f4v n4 = ht4(Md::B_HFACE + 4 * (f > 0 ? f : 0));
      const float nf[3] = {-n4.x, -n4.y, -n4.z};
      float sv[3];
      side(mp - 1, sv);
      for (int a = 0; a < 3; a++) mu[a] = mp == 0 ? ntm[a] : (mp < 4 ? sv[a] : (mp == 4 ? -zc[a] : nf[a]));
    }
    // the contact point: hull vertices inside the prism and prism top vertices inside the hull,
    // weighted by their penetration
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 13
    for (int rep_ = 0; rep_ < 2; rep_++) {
      float Tm_l[3][3], sm_l[3][3], ntm_l[3] = {ntm[0], ntm[1], ntm[2]}, zc_l[3] = {zc[0], zc[1], zc[2]};
      float mu_l[3] = {mu[0], mu[1], mu[2]};
      for (int k = 0; k < 3; k++)
        for (int a = 0; a < 3; a++) Tm_l[k][a] = Tm[k][a], sm_l[k][a] = sm[k][a];
      launder<9>(&Tm_l[0][0]);
      launder<9>(&sm_l[0][0]);
      launder<3>(ntm_l);
      launder<3>(zc_l);
      launder<3>(mu_l);
      const auto& Tm = Tm_l;
      const auto& sm = sm_l;
      const auto& ntm = ntm_l;
      const auto& zc = zc_l;
      const auto& mu = mu_l;
#endif
    const float ptop = dot3(ntm, Tm[0]);
    const float smt[3] = {dot3(sm[0], Tm[0]), dot3(sm[1], Tm[1]), dot3(sm[2], Tm[2])};
    float W = 0.0f, Cx[3] = {0.0f, 0.0f, 0.0f};
    // (every vertex, without a wave-uniform skip of those above every lane's prism top: the 17
    // branches cost more than the distances they skipped, C4 -0.8 %; the weights are the same)
    static_for<0, NH>([&](auto kI) {
      constexpr int k = kI.value;
      // (o - v_k . x with the offset fused into the first product, v_fmamk_f32, measured C4 +0.7 % and
      // C5 +0.9 %, but moved the teacher-forced outliers: rough + DR seeds 7 / 11 / 13 / 17 10 / 24 /
      // 16 / 12 of 10,240 with one unexplained, against 13 / 20 / 14 / 13 all explained -- not kept)
      float d[5];
      hv_dot5<k>(ntm, zc, sm[0], sm[1], sm[2], d);
      const float atop = ptop - d[0];
      float pen = fminf(atop, d[1] - base);
      for (int j = 0; j < 3; j++) pen = fminf(pen, smt[j] - d[2 + j]);
      const float w = fmaxf(pen, 0.0f);
      W += w;
      Cx[0] = cfma<fbits(Md::hull_vert[k][0])>(w, Cx[0]);
      Cx[1] = cfma<fbits(Md::hull_vert[k][1])>(w, Cx[1]);
      Cx[2] = cfma<fbits(Md::hull_vert[k][2])>(w, Cx[2]);
    });
    {
      // the prism's top vertices inside the hull: the faces in HullFaceOrder, and once no lane of the
      // wave has a vertex still inside every face tested so far (checked after the first 6 and 14),
      // the rest are skipped -- every weight is 0 then, and the minimum is order-independent
      float pk[3] = {1e30f, 1e30f, 1e30f};
      bool live = true;
      static_for<0, NF>([&](auto pI) {
        constexpr int pos = pI.value;
        constexpr int f = HullFaceOrder<Md>{}.f[pos];
        if (pos == 6 || pos == 14) live = live && __ballot(fmaxf(pk[0], fmaxf(pk[1], pk[2])) > 0.0f) != 0ull;
        if (!live) return;
        float d[3];
        nf_off_dot3<f>(Tm[0], Tm[1], Tm[2], d);
#pragma unroll
        for (int j = 0; j < 3; j++) pk[j] = fminf(pk[j], d[j]);
      });
#pragma unroll
      for (int j = 0; j < 3; j++) {
        const float w = fmaxf(pk[j], 0.0f);
        W += w;
        for (int a = 0; a < 3; a++) Cx[a] += w * Tm[j][a];
      }
    }
    float pos[3];
    if (W > 0.0f) {
      const float iw = 1.0f / W;
      for (int a = 0; a < 3; a++) pos[a] = Cx[a] * iw;
    } else {
      // no vertex inside at all (crossing edges): the midpoint of the two shapes' support features
      // along mu. (Round 4 blended towards it below a total weight of 1e-4 m -- a "point band" for
      // onset prisms; fp32 and fp64 then disagreed 2-3x as often)
      float hmu = 1e30f;
      float hv[NH];
      static_for<0, NH>([&](auto kI) { hv[kI.value] = hv_dot<kI.value>(mu); });
#pragma unroll
      for (int k = 0; k < NH; k++) hmu = fminf(hmu, hv[k]);
      float wh_ = 0.0f, ch[3] = {0.0f, 0.0f, 0.0f};
      static_for<0, NH>([&](auto kI) {
        constexpr int k = kI.value;
        const float w = fmaxf(0.0f, 1.0f - (hv[k] - hmu) * (1.0f / HF_WITNESS_BAND));
        wh_ += w;
        ch[0] = cfma<fbits(Md::hull_vert[k][0])>(w, ch[0]);
        ch[1] = cfma<fbits(Md::hull_vert[k][1])>(w, ch[1]);
        ch[2] = cfma<fbits(Md::hull_vert[k][2])>(w, ch[2]);
      });
      const float q[3] = {dot3(mu, Tm[0]), dot3(mu, Tm[1]), dot3(mu, Tm[2])};
      const float pmx = fmaxf(q[0], fmaxf(q[1], q[2]));
      float wp_ = 0.0f, cq[3] = {0.0f, 0.0f, 0.0f};
      for (int k = 0; k < 3; k++) {
        const float w = fmaxf(0.0f, 1.0f - (pmx - q[k]) * (1.0f / HF_WITNESS_BAND));
        wp_ += w;
        for (int a = 0; a < 3; a++) cq[a] += w * Tm[k][a];
      }
      const float iwh = frcp(wh_), iwp = frcp(wp_);
      for (int a = 0; a < 3; a++) pos[a] = 0.5f * (ch[a] * iwh + cq[a] * iwp);
    }
    E4[0] = f4v{mo, mu[0], mu[1], mu[2]};
    E4[1] = f4v{pos[0], pos[1], pos[2], 0.0f};
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 13
    }
#endif
  }

  // the grid offsets (column, row) of top vertex k of a cell's triangle: A (tri 0) = (0, 0), (0, 1), (1, 0);
  // B (tri 1) = (0, 1), (1, 0), (1, 1). Arithmetic on tri: written as a table indexed by tri the compiler
  // made it a lookup in global memory, two dependent loads per prism slot in the survivor descriptors
  static DK int tri_dc(int k, int tri) { return k == 0 ? 0 : (k == 1 ? tri : 1); }
  static DK int tri_dr(int k, int tri) { return k == 0 ? tri : (k == 1 ? 1 - tri : tri); }

  static DK void collide_hfield(LP L, int lane, const float* hf) {
    STAGE_T0();
    constexpr int NH = Md::NHV, NF = Md::NHF, NE = Md::NHE;
    constexpr int NR = Md::HF_NROW, NCc = Md::HF_NCOL;
    constexpr float SX = Md::HF_SIZE[0], SY = Md::HF_SIZE[1], SZ = Md::HF_SIZE[2], SB = Md::HF_SIZE[3];
    constexpr float DXC = 2.0f * SX / (NCc - 1), DYC = 2.0f * SY / (NR - 1);
    constexpr int MAXP = 2 * Md::HF_MAXCX * Md::HF_MAXCY, PPL = (MAXP + 7) / 8;
    static_assert(MAXP <= 32, "prism masks are 32-bit");
    constexpr int NGV = (Md::HF_MAXCX + 1) * (Md::HF_MAXCY + 1), GPL = (NGV + 7) / 8;
    constexpr int VPL = (NH + 7) / 8, FPL = (NF + 7) / 8, EPL = (NE + 7) / 8;
    const int h = lane >> 3, sub = lane & 7;
    const int p = Md::PLANE_PAIR[0] * (1 - h) + Md::PLANE_PAIR[1] * h;
    const int gs = cgeom_slot<Md>(Md::pair_geom2[p]);
    float pp[3], PR[9], cp[3], CR[9];
    S1 Ls{L};
    P1::geom_frame(Ls, 0, pp, PR);
    cgeom_frame(L, gs, cp, CR);
    float R[9], t[3];  // mesh -> local rotation; the hull frame's origin in the field frame
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) R[3 * a + b] = PR[a] * CR[b] + PR[3 + a] * CR[3 + b] + PR[6 + a] * CR[6 + b];
    {
      const float d[3] = {cp[0] - pp[0], cp[1] - pp[1], cp[2] - pp[2]};
      mulmtv3(t, PR, d);
    }
    const float zc[3] = {R[6], R[7], R[8]};  // the field's z axis in the mesh frame
    // this lane's hull vertices (local) and the hull's bounding box
    float xl[VPL][3];
    bool vok[VPL];
    float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
    const float GN = 1.0f / sqrtf(DXC * DXC + DYC * DYC);
    const float GX = DYC * GN, GY = DXC * GN;  // the cells' diagonal side normal (dy, dx) / |.|
#pragma unroll
    for (int i = 0; i < VPL; i++) {
      const int k = sub + 8 * i;
      vok[i] = k < NH;
      const int kk = vok[i] ? k : 0;
      const float v[3] = {tf(Md::B_HULL + 3 * kk), tf(Md::B_HULL + 3 * kk + 1), tf(Md::B_HULL + 3 * kk + 2)};
      mulmv3(xl[i], R, v);
      if (vok[i]) {
        for (int a = 0; a < 3; a++) { lo[a] = fminf(lo[a], xl[i][a]); hi[a] = fmaxf(hi[a], xl[i][a]); }
      }
    }
    for (int a = 0; a < 3; a++) { lo[a] = hmin8f(lo[a]); hi[a] = hmax8_nc(hi[a]); }
    // the field's box and the sub-grid (vertex columns cmin..cmax, rows rmin..rmax); grid
    // coordinates relative to the field's centre (vertex c at (c - (ncol - 1) / 2) dx): the robot
    // walks near the centre, where these keep fp32's resolution (x + size would round to ~1e-6 m)
    const bool inside = !(hi[0] + t[0] < -SX || lo[0] + t[0] > SX || hi[1] + t[1] < -SY || lo[1] + t[1] > SY ||
                          lo[2] + t[2] > SZ || hi[2] + t[2] < -SB);
    constexpr float FXC = (NCc - 1) / (2.0f * SX), FYC = (NR - 1) / (2.0f * SY);
    constexpr float CC0 = 0.5f * (NCc - 1), RC0 = 0.5f * (NR - 1);
    const int cmin = max((int)floorf((lo[0] + t[0]) * FXC + CC0), 0);
    const int cmax = min((int)ceilf((hi[0] + t[0]) * FXC + CC0), NCc - 1);
    const int rmin = max((int)floorf((lo[1] + t[1]) * FYC + RC0), 0);
    const int rmax = min((int)ceilf((hi[1] + t[1]) * FYC + RC0), NR - 1);
    const int ncx = inside ? min(max(cmax - cmin, 0), Md::HF_MAXCX) : 0;
    const int ncy = inside ? min(max(rmax - rmin, 0), Md::HF_MAXCY) : 0;
    const int np = 2 * ncx * ncy;
    const float X0 = ((float)cmin - CC0) * DXC - t[0], Y0 = ((float)rmin - RC0) * DYC - t[1];
    const float base = -SB - t[2];  // the prisms' bottom (local z)
    // the sub-grid's elevations (local z), one global load per lane: vertex v = iy (ncx + 1) + ix
    // on lane v & 7, register v >> 3; prisms read them by shuffles. The loads are unconditional (an
    // in-range index on every lane) and issue here, back to back; the side minima and the silhouette
    // lists run before their first use (as conditional loads each waited for itself at once: two
    // exposed L2 round trips per substep)
    float zg[GPL], hraw[GPL];
    bool zok[GPL];
#pragma unroll
    for (int i = 0; i < GPL; i++) {
      const int v = sub + 8 * i, iy = v / (ncx + 1), ix = v - iy * (ncx + 1);
      zok[i] = np > 0 && iy <= ncy;
      hraw[i] = hf[zok[i] ? (rmin + iy) * NCc + cmin + ix : 0];
    }
    auto zat = [&](int ix, int iy) -> float {  // any lane pattern: every lane supplies both registers
      const int v = iy * (ncx + 1) + ix, src = 8 * h + (v & 7);
      float z = __shfl(zg[0], src, TEAM);
#pragma unroll
      for (int i = 1; i < GPL; i++) {
        const float zi = __shfl(zg[i], src, TEAM);
        z = (v >> 3) == i ? zi : z;
      }
      return z;
    };
    // prism q (strip order): cell (rr, cc) of the sub-grid, triangle tri; top vertices (local)
    // A = (c, r), (c, r + 1), (c + 1, r); B = (c, r + 1), (c + 1, r), (c + 1, r + 1)
    auto prism_top = [&](int q, float (*T)[3], int& tri) {
      const int rr = q / (2 * ncx), rem = q - rr * 2 * ncx, cc = rem >> 1;
      tri = rem & 1;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        const int ci = cc + tri_dc(k, tri), ri = rr + tri_dr(k, tri);
        T[k][0] = X0 + (float)ci * DXC;
        T[k][1] = Y0 + (float)ri * DYC;
        T[k][2] = zat(ci, ri);
      }
    };
    auto top_normal = [&](const float (*T)[3], float* nt) {
      const float e0[3] = {T[1][0] - T[0][0], T[1][1] - T[0][1], T[1][2] - T[0][2]};
      const float e1[3] = {T[2][0] - T[0][0], T[2][1] - T[0][1], T[2][2] - T[0][2]};
      cross3(nt, e0, e1);
      const float sg = (nt[2] < 0.0f ? -1.0f : 1.0f) / sqrtf(dot3(nt, nt));
      for (int a = 0; a < 3; a++) nt[a] *= sg;
    };
    // the hull's lowest point along each side normal (the six directions of the two triangle kinds:
    // A (-x, +g, -y), B (-g, +x, +y))
    const float sx_[2][3] = {{-1.0f, GX, 0.0f}, {-GX, 1.0f, 0.0f}}, sy_[2][3] = {{0.0f, GY, -1.0f}, {-GY, 0.0f, 1.0f}};
    float smin[2][3];
#pragma unroll
    for (int ty = 0; ty < 2; ty++)
#pragma unroll
      for (int k = 0; k < 3; k++) {
        float mv = 1e30f;
#pragma unroll
        for (int i = 0; i < VPL; i++)
          if (vok[i]) mv = fminf(mv, sx_[ty][k] * xl[i][0] + sy_[ty][k] * xl[i][1]);
        smin[ty][k] = hmin8f(mv);
      }
    const float obot = hi[2] - base;
    // this foot's silhouette edges (the hull's edges whose faces straddle the field's horizontal
    // plane: the only ones whose Gauss arc crosses a prism's vertical-edge arc), compacted in edge
    // order into the env slice's composite-inertia storage (dead after crb()): the direction w in
    // which the negated arc crosses the equator and the hull's support along it
    lds_float* const SLo = L + HF_CINQ + h * HF_SLSZ;
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 17
    for (int rep_ = 0; rep_ < 2; rep_++)
#endif
    {
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 17
      float zc_l[3] = {zc[0], zc[1], zc[2]};
      launder<3>(zc_l);
      const auto& zc = zc_l;
#endif
      unsigned long long M = 0;
      float wv[EPL][3], wh[EPL];
      bool sl[EPL];
#pragma unroll
      for (int j = 0; j < EPL; j++) {
        const int e = sub + 8 * j, ee = e < NE ? e : 0, o = Md::B_HEDGE + 20 * ee;
        const f4v C4 = ht4(o), D4 = ht4(o + 4), v04 = ht4(o + 16);
        const float C[3] = {C4.x, C4.y, C4.z}, D[3] = {D4.x, D4.y, D4.z}, v0[3] = {v04.x, v04.y, v04.z};
        const float sa = dot3(C, zc), sb = dot3(D, zc);
        const float w[3] = {fabsf(sb) * C[0] + fabsf(sa) * D[0], fabsf(sb) * C[1] + fabsf(sa) * D[1],
                            fabsf(sb) * C[2] + fabsf(sa) * D[2]};
        const float wn = sqrtf(dot3(w, w));
        sl[j] = e < NE && sa * sb < 0.0f && wn > 0.0f;
        const float inv = sl[j] ? frcp(wn) : 0.0f;  // (1.0f / wn compiled to the correctly rounded division)
        for (int a = 0; a < 3; a++) wv[j][a] = w[a] * inv;
        wh[j] = dot3(wv[j], v0);
        M |= (unsigned long long)half_bits(__ballot(sl[j]), lane) << (8 * j);
      }
#pragma unroll
      for (int j = 0; j < EPL; j++) {
        const int e = sub + 8 * j;
        const int r = __popcll(M & ((1ull << e) - 1ull));
        if (sl[j] && r < Md::HF_SILCAP) {
          ((lds_int*)SLo)[1 + r] = e;
          ((lds_f4*)(SLo + HF_SLF))[r] = f4v{wv[j][0], wv[j][1], wv[j][2], wh[j]};
        }
      }
      if (sub == 0) ((lds_int*)SLo)[0] = min(__popcll(M), Md::HF_SILCAP);
    }
#pragma unroll
    for (int i = 0; i < GPL; i++) zg[i] = zok[i] ? SZ * hraw[i] - t[2] : 0.0f;
    // 1. lane-parallel screen: prism q = sub + 8 j passes the height test and the axes of its own
    // faces, the bottom and the hull's faces (the hull's support along its top normal from the
    // compile-time vertices). The running minimum and its axis priority are kept: the survivors'
    // SAT (hf_exec) continues from them with the edge pairs.
    float smo[PPL], szt[PPL][3];
    int smp[PPL];
    unsigned surv = 0;
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 14
    for (int rep_ = 0; rep_ < 2; rep_++) {
      launder<9>(R);
      launder<GPL>(zg);
      launder<3>(lo);
#endif
#pragma unroll
    for (int j = 0; j < PPL; j++) {
      const int q = sub + 8 * j;
      smo[j] = 0.0f;
      smp[j] = 0;
      for (int k = 0; k < 3; k++) szt[j][k] = 0.0f;
      // (a wave-uniform skip of the slots no foot of the wave has: most sub-grids hold <= 12 prisms)
      if (j > 0 && __ballot(q < np) == 0ull) continue;
      float T[3][3], nt[3];
      int tri;
      prism_top(q < np ? q : 0, T, tri);
      top_normal(T, nt);
      float ntm[3];
      mulmtv3(ntm, R, nt);
      float hm = 1e30f;
      // (vertex pairs: two interleaved products per statement; the minimum is order-independent)
      static_for<0, NH / 2>([&](auto kI) {
        float ha, hb;
        hv_dot2<2 * kI.value>(ntm, ha, hb);
        hm = fmin_nc(hm, fmin_nc(ha, hb));
      });
      if constexpr (NH % 2) hm = fminf(hm, hv_dot<NH - 1>(ntm));
      // priority order (equal overlaps: the first): top 0, sides 1-3, bottom 4, hull faces 5 + f
      float mo = dot3(nt, T[0]) - hm;
      int mp = 0;
      for (int k = 0; k < 3; k++) {  // (tri is 0 or 1: two-way selects, not an indexed register array)
        const float sxk = tri ? sx_[1][k] : sx_[0][k], syk = tri ? sy_[1][k] : sy_[0][k];
        const float ov = sxk * T[k][0] + syk * T[k][1] - (tri ? smin[1][k] : smin[0][k]);
        mp = ov < mo ? 1 + k : mp;
        mo = fminf(mo, ov);
      }
      mp = obot < mo ? 4 : mp;
      mo = fminf(mo, obot);
      // (the hull's 30 face axes are the survivors' first SAT step, hf_exec: per survivor lane once,
      // instead of per screened prism slot -- they separate ≈ 0.6 prisms per foot-substep more)
      const bool high = !(T[0][2] < lo[2] && T[1][2] < lo[2] && T[2][2] < lo[2]);
      const bool ok = q < np && high && mo > 0.0f;
      surv |= half_bits(__ballot(ok), lane) << (8 * j);
      smo[j] = mo;
      smp[j] = mp;
      for (int k = 0; k < 3; k++) szt[j][k] = T[k][2];
    }
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 14
    }
#endif
    float cd[PPL], cn[PPL][3], cx[PPL][3];  // this lane's prism contacts: depth, normal, point (local)
#pragma unroll
    for (int s = 0; s < PPL; s++) {
      cd[s] = -1.0f;
      for (int a = 0; a < 3; a++) { cn[s][a] = 0.0f; cx[s][a] = 0.0f; }
    }
    STAGE_MARK(37);
    // 2. the survivors of the wave's 8 feet, one per lane: a queue in the H + constraint-row
    // storage of the wave's 4 env slices (dead until make_rows()), entry g in slice g & 3; each
    // lane writes its survivors' descriptors (mesh frame), every active lane runs one entry's SAT
    // (hf_exec) and writes the contact back, the owners collect them. Rounds of QR entries.
    const int hw = ((int)threadIdx.x & 63) >> 3, tw = hw >> 1;
    const unsigned long long act = __ballot(1);
    int S = 0, g0 = 0;
    {
      const int cnt = __popc(surv);
#pragma unroll
      for (int hh = 0; hh < 8; hh++) {
        const int c = ((act >> (8 * hh)) & 1ull) ? __builtin_amdgcn_readlane(cnt, 8 * hh) : 0;
        g0 += hh < hw ? c : 0;
        S += c;
      }
    }
    const int nact = __popcll(act), QRa = nact < HF_QR ? nact : HF_QR;
#ifdef DUCK_STAGE_PROF
    if (threadIdx.x == 0) STAGE_ADD(40, (unsigned long long)S);
    // the survivors' distribution over wave-substeps (wave 0): <= 21, 22-32, 33-42, 43-64, > 64
    if (threadIdx.x == 0) STAGE_ADD(S <= 21 ? 51 : (S <= 32 ? 52 : (S <= 42 ? 53 : (S <= 64 ? 54 : 55))), 1ull);
#endif
    const int gi = __popcll(act & ((1ull << ((int)threadIdx.x & 63)) - 1ull));  // this lane among the active
    auto qent = [&](int g) -> lds_float* { return L + ((g & 3) - tw) * TL::STRIDE + HF_QH0 + HF_ENT * (g >> 2); };
    for (int r0 = 0; r0 < S; r0 += QRa) {
#ifdef DUCK_STAGE_PROF
      if (threadIdx.x == 0) STAGE_ADD(46, 1ull);
#endif
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 18
      for (int rep_ = 0; rep_ < 2; rep_++) {
      launder<9>(R);
#endif
#pragma unroll
      for (int j = 0; j < PPL; j++) {
        const int q = sub + 8 * j;
        const int g = g0 + __popc(surv & ((1u << q) - 1u)) - r0;
        const bool mine = ((surv >> q) & 1u) && g >= 0 && g < QRa;
        if (__ballot(mine) == 0ull) continue;
        if (mine) {
          // the prism's top (local) as the screen had it, then the mesh frame
          const int rr = q / (2 * ncx), rem = q - rr * 2 * ncx, cc = rem >> 1, tri = rem & 1;
          float T[3][3], nt[3], ntm[3], Tm[3][3];
#pragma unroll
          for (int k = 0; k < 3; k++) {
            T[k][0] = X0 + (float)(cc + tri_dc(k, tri)) * DXC;
            T[k][1] = Y0 + (float)(rr + tri_dr(k, tri)) * DYC;
            T[k][2] = szt[j][k];
          }
          top_normal(T, nt);
          mulmtv3(ntm, R, nt);
          for (int k = 0; k < 3; k++) mulmtv3(Tm[k], R, T[k]);
          lds_f4* E4 = (lds_f4*)qent(g);
          E4[0] = f4v{Tm[0][0], Tm[0][1], Tm[0][2], base};
          E4[1] = f4v{Tm[1][0], Tm[1][1], Tm[1][2], smo[j]};
          E4[2] = f4v{Tm[2][0], Tm[2][1], Tm[2][2], __int_as_float(smp[j])};
          E4[3] = f4v{ntm[0], ntm[1], ntm[2], __int_as_float(tri | (2 * tw + h) << 1)};
          E4[4] = f4v{zc[0], zc[1], zc[2], szt[j][0]};
          E4[5] = f4v{R[0], R[1], R[2], szt[j][1]};
          E4[6] = f4v{R[3], R[4], R[5], szt[j][2]};
        }
      }
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 18
      }
#endif
      TSYNC();
      STAGE_MARK(41);
#ifdef DUCK_ASM_MARKS
      asm volatile("; HF_EXEC_BEGIN" ::: "memory");
#endif
      if (gi < QRa && r0 + gi < S) hf_exec(qent(gi), L, tw);
#ifdef DUCK_ASM_MARKS
      asm volatile("; HF_EXEC_END" ::: "memory");
#endif
      TSYNC();
      STAGE_MARK(42);
#pragma unroll
      for (int j = 0; j < PPL; j++) {
        const int q = sub + 8 * j;
        const int g = g0 + __popc(surv & ((1u << q) - 1u)) - r0;
        const bool mine = ((surv >> q) & 1u) && g >= 0 && g < QRa;
        if (__ballot(mine) == 0ull) continue;
        if (mine) {
          const lds_f4* O = (const lds_f4*)qent(g);
          const f4v o0 = O[0], o1 = O[1];
          const float um[3] = {o0.y, o0.z, o0.w}, pm[3] = {o1.x, o1.y, o1.z};
          cd[j] = o0.x > 0.0f ? o0.x : -1.0f;
          mulmv3(cn[j], R, um);
          mulmv3(cx[j], R, pm);
        }
      }
      TSYNC();
      STAGE_MARK(43);
    }
    STAGE_MARK(38);
    // 4 slots by mjx's _manifold_points over the prism contacts, from the deepest (the first prism
    // within HF_DEPTH_TIE of it: prisms sharing a grid vertex or edge often tie exactly); index
    // q = sub + 8 s is the prism's strip position
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 19
    for (int rep_ = 0; rep_ < 2; rep_++) {
    launder<PPL>(cd);
    launder<3 * PPL>(&cx[0][0]);
    launder<3 * PPL>(&cn[0][0]);
#endif
    constexpr int QN = 8 * PPL;
    float dmax = -1e30f;
#pragma unroll
    for (int s = 0; s < PPL; s++) dmax = fmaxf(dmax, cd[s] > 0.0f ? cd[s] : -1e30f);
    dmax = hmax8_nc(dmax);
    const bool any = dmax > 0.0f;
    int a_ = 1 << 20;
#pragma unroll
    for (int s = PPL - 1; s >= 0; s--)
      a_ = ((cd[s] > 0.0f) & (cd[s] >= dmax - HF_DEPTH_TIE)) ? sub + 8 * s : a_;  // (& : selects, not branches)
    a_ = hmin8i(a_);
    a_ = a_ < QN ? a_ : 0;
    // a contact's fields, fetched from its owner lane (q uniform over the half-team)
    auto fetch = [&](int q, float* x, float* n, float& d) {
      float px[3], pn[3], pd = cd[0];
      for (int a = 0; a < 3; a++) { px[a] = cx[0][a]; pn[a] = cn[0][a]; }
#pragma unroll
      for (int s = 1; s < PPL; s++) {
        const bool m = (q >> 3) == s;
        pd = m ? cd[s] : pd;
        for (int a = 0; a < 3; a++) { px[a] = m ? cx[s][a] : px[a]; pn[a] = m ? cn[s][a] : pn[a]; }
      }
      const int src = 8 * h + (q & 7);
      d = __shfl(pd, src, TEAM);
      for (int a = 0; a < 3; a++) { x[a] = __shfl(px[a], src, TEAM); n[a] = __shfl(pn[a], src, TEAM); }
    };
    // argmax with mjx's tolerance: the first index within tol of the maximum (valid contacts only)
    auto argmax = [&](const float* v, float tol) -> int {
      float mx = -1e30f;
#pragma unroll
      for (int s = 0; s < PPL; s++) mx = fmaxf(mx, v[s]);
      mx = hmax8_nc(mx);
      int best = 1 << 20;
#pragma unroll
      for (int s = PPL - 1; s >= 0; s--)
        best = ((cd[s] > 0.0f) & (v[s] >= mx - tol)) ? sub + 8 * s : best;
      best = hmin8i(best);
      return best < QN ? best : a_;
    };
    float pa[3], na[3], da, sc[PPL];
    fetch(a_, pa, na, da);
#pragma unroll
    for (int s = 0; s < PPL; s++) {
      const float dx = pa[0] - cx[s][0], dy = pa[1] - cx[s][1], dz = pa[2] - cx[s][2];
      sc[s] = cd[s] > 0.0f ? dx * dx + dy * dy + dz * dz : -1e30f;
    }
    const int b_ = argmax(sc, MANIFOLD_TOL);
    float pb[3], nb[3], db;
    fetch(b_, pb, nb, db);
    float ab[3];
    {
      const float amb[3] = {pa[0] - pb[0], pa[1] - pb[1], pa[2] - pb[2]};
      cross3(ab, na, amb);
    }
#pragma unroll
    for (int s = 0; s < PPL; s++) {
      const float ap[3] = {pa[0] - cx[s][0], pa[1] - cx[s][1], pa[2] - cx[s][2]};
      sc[s] = cd[s] > 0.0f ? fabsf(dot3(ap, ab)) : -1e30f;
    }
    const int c_ = argmax(sc, MANIFOLD_TOL);
    float pc[3], nc_[3], dcc;
    fetch(c_, pc, nc_, dcc);
    float ac[3], bc[3];
    {
      const float amc[3] = {pa[0] - pc[0], pa[1] - pc[1], pa[2] - pc[2]};
      const float bmc[3] = {pb[0] - pc[0], pb[1] - pc[1], pb[2] - pc[2]};
      cross3(ac, na, amc);
      cross3(bc, na, bmc);
    }
    int d_;
    {
      float s1[PPL], s2[PPL], mx = -1e30f;
#pragma unroll
      for (int s = 0; s < PPL; s++) {
        const float bp[3] = {pb[0] - cx[s][0], pb[1] - cx[s][1], pb[2] - cx[s][2]};
        const float ap[3] = {pa[0] - cx[s][0], pa[1] - cx[s][1], pa[2] - cx[s][2]};
        s1[s] = cd[s] > 0.0f ? fabsf(dot3(bp, bc)) : -1e30f;
        s2[s] = cd[s] > 0.0f ? fabsf(dot3(ap, ac)) : -1e30f;
        mx = fmaxf(mx, fmaxf(s1[s], s2[s]));
      }
      mx = hmax8_nc(mx);
      int best = 1 << 20;
#pragma unroll
      for (int s = PPL - 1; s >= 0; s--) {
        best = ((cd[s] > 0.0f) & (s2[s] >= mx - MANIFOLD_TOL)) ? QN + sub + 8 * s : best;
      }
#pragma unroll
      for (int s = PPL - 1; s >= 0; s--) {
        best = ((cd[s] > 0.0f) & (s1[s] >= mx - MANIFOLD_TOL)) ? sub + 8 * s : best;
      }
      d_ = hmin8i(best);
      d_ = d_ < 2 * QN ? (d_ >= QN ? d_ - QN : d_) : a_;
    }
    // slot sub (< 4) of this pair: its contact, repeats inactive (fetches are uniform over the
    // half-team: a lane's shuffle source selects its slot with the requester's index)
    float pdd[3], ndd[3], ddd;
    fetch(d_, pdd, ndd, ddd);
    // slot sub's contact by v_cndmask on the lanes' sub masks: written as nested ?: on sub, the compiler
    // made each of the seven values a tree of exec-masked branches
    const unsigned long long m0 = __ballot(sub == 0), m1 = __ballot(sub == 1), m2 = __ballot(sub == 2);
    auto pick = [&](float v0, float v1, float v2, float v3) { return vsel(m0, v0, vsel(m1, v1, vsel(m2, v2, v3))); };
    const int myq = (sub == 0) * a_ + (sub == 1) * b_ + (sub == 2) * c_ + (sub >= 3) * d_;
    float px[3], pn[3], pd;
    for (int a = 0; a < 3; a++) {
      px[a] = pick(pa[a], pb[a], pc[a], pdd[a]);
      pn[a] = pick(na[a], nb[a], nc_[a], ndd[a]);
    }
    pd = pick(da, db, dcc, ddd);
    if (sub < 4) {
      const int idx[4] = {a_, b_, c_, d_};
      bool unique = true;
      for (int e = 0; e < 4; e++) unique = unique & !((e < sub) & (idx[e] == myq));
      float fr[9], pw[3], nw[3];
      if (any) {
        const float pl[3] = {px[0] + t[0], px[1] + t[1], px[2] + t[2]};
        mulmv3(pw, PR, pl);
        for (int a = 0; a < 3; a++) pw[a] += pp[a];
        mulmv3(nw, PR, pn);
        make_frame(fr, nw);
        P1::store_contact(Ls, 4 * p + sub, unique ? -pd : 1.0f, pw, fr);
      } else {
        const float nofr[9] = {0, 0, 1, 0, 1, 0, -1, 0, 0};
        const float zero[3] = {L[Ly::COM], L[Ly::COM + 1], L[Ly::COM + 2]};
        P1::store_contact(Ls, 4 * p + sub, 1.0f, zero, nofr);
      }
    }
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 19
    }
#endif
    STAGE_MARK(39);
  }

  // Are the boxes enclosing the two hulls (mesh frames p, R) separated? 15-axis box/box SAT
  // (face axes of both boxes and their 9 edge-pair axes), with a 1e-5 m margin so that only a
  // clear separation rejects: then the hulls inside are separated too and the full hull SAT
  // would report no contact.
  static DK bool boxes_separated(const float* p1, const float* R1, const float* p2, const float* R2) {
    const float* h = Md::hull_box_h;
    float c1[3], c2[3], t[3], T[3], Ta[3], Rr[3][3], Ar[3][3];
    mulmv3(t, R1, Md::hull_box_c);
    for (int k = 0; k < 3; k++) c1[k] = p1[k] + t[k];
    mulmv3(t, R2, Md::hull_box_c);
    for (int k = 0; k < 3; k++) c2[k] = p2[k] + t[k];
    for (int k = 0; k < 3; k++) T[k] = c2[k] - c1[k];
    mulmtv3(Ta, R1, T);  // center offset in box 1's axes
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {  // Rr[i][j] = axis i of box 1 . axis j of box 2
        Rr[i][j] = R1[i] * R2[j] + R1[3 + i] * R2[3 + j] + R1[6 + i] * R2[6 + j];
        Ar[i][j] = fabsf(Rr[i][j]) + 1e-6f;
      }
    constexpr float MARGIN = 1e-5f;
    bool sep = false;
    for (int i = 0; i < 3; i++)
      sep = sep || fabsf(Ta[i]) > h[i] + h[0] * Ar[i][0] + h[1] * Ar[i][1] + h[2] * Ar[i][2] + MARGIN;
    for (int j = 0; j < 3; j++) {
      const float tb = Ta[0] * Rr[0][j] + Ta[1] * Rr[1][j] + Ta[2] * Rr[2][j];
      sep = sep || fabsf(tb) > h[j] + h[0] * Ar[0][j] + h[1] * Ar[1][j] + h[2] * Ar[2][j] + MARGIN;
    }
    for (int i = 0; i < 3; i++) {
      const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
      for (int j = 0; j < 3; j++) {
        const int j1 = (j + 1) % 3, j2 = (j + 2) % 3;
        const float ra = h[i1] * Ar[i2][j] + h[i2] * Ar[i1][j];
        const float rb = h[j1] * Ar[i][j2] + h[j2] * Ar[i][j1];
        sep = sep || fabsf(Ta[i2] * Rr[i1][j] - Ta[i1] * Rr[i2][j]) > ra + rb + MARGIN;
      }
    }
    return sep;
  }

  // Hull/hull (foot/foot) SAT with the team: mjx / oracle collide_convex_convex semantics, the
  // axes split over the lanes, then mjx's clipped face manifold or the edge pair's closest points. Face axes (both hulls, 60) then edge-pair axes (45 x 45); a
  // separating axis anywhere means no contact (the 4 slots stay inactive); otherwise the best
  // face (largest separation, first index among equal ones) unless the best edge pair beats it
  // by 1e-9 (declared deviation: the single-lane scan applies that margin per step, here it is
  // applied to the edges' maximum). Vertices and edge directions in world coordinates are kept
  // in registers (vertices) and in the dead H / constraint-row storage (edges).
  static DK void collide_hulls_team(LP L, int lane, int slot0, const float* p1, const float* R1, const float* p2,
                                    const float* R2, const float* cc) {
    constexpr int NH = Md::NHV, NF = Md::NHF, NE = Md::NHE;
    constexpr int EA = Ly::H, EB = EA + 3 * NE;
    static_assert(EB + 3 * NE <= Ly::CR, "edge scratch must fit in the H / row storage");
    S1 Ls{L};
    if (lane < 4) {
      const float nofr[9] = {0, 0, 1, 0, 1, 0, -1, 0, 0};
      const float zero[3] = {L[Ly::COM], L[Ly::COM + 1], L[Ly::COM + 2]};
      P1::store_contact(Ls, slot0 + lane, 1.0f, zero, nofr);
    }
    float V1[NH][3], V2[NH][3], t[3];
#pragma unroll
    for (int k = 0; k < NH; k++) {
      const float v[3] = {tf(Md::B_HULL + 3 * k), tf(Md::B_HULL + 3 * k + 1), tf(Md::B_HULL + 3 * k + 2)};
      mulmv3(t, R1, v);
      for (int q = 0; q < 3; q++) V1[k][q] = p1[q] + t[q];
      mulmv3(t, R2, v);
      for (int q = 0; q < 3; q++) V2[k][q] = p2[q] + t[q];
    }
    const int(*HE)[2] = Md::hull_edge_d();
    const int(*HEF)[2] = Md::hull_edge_face_d();
    const float(*HN)[3] = Md::hull_face_normal_d();
    // world face normals: hull 1 as is, hull 2 negated (the Gauss map of -B, whose faces are
    // also the face axes of side 1)
    constexpr int FA = EB + 3 * NE, FB = FA + 3 * NF;
    static_assert(FB + 3 * NF <= Ly::CR, "face-normal scratch must fit in the H / row storage");
    for (int e = lane; e < NE; e += TEAM) {
      const int a0 = HE[e][0], a1 = HE[e][1];
      float d[3];
      for (int q = 0; q < 3; q++) d[q] = tf(Md::B_HULL + 3 * a1 + q) - tf(Md::B_HULL + 3 * a0 + q);
      mulmv3(t, R1, d);
      for (int q = 0; q < 3; q++) L[EA + 3 * e + q] = t[q];
      mulmv3(t, R2, d);
      for (int q = 0; q < 3; q++) L[EB + 3 * e + q] = t[q];
    }
    for (int f = lane; f < NF; f += TEAM) {
      mulmv3(t, R1, HN[f]);
      for (int q = 0; q < 3; q++) L[FA + 3 * f + q] = t[q];
      mulmv3(t, R2, HN[f]);
      for (int q = 0; q < 3; q++) L[FB + 3 * f + q] = -t[q];
    }
    TSYNC();
    auto sep_of = [&](const float* u) {
      float mx1 = -1e30f, mn2 = 1e30f;
#pragma unroll
      for (int k = 0; k < NH; k++) {
        mx1 = fmaxf(mx1, dot3(u, V1[k]));
        mn2 = fminf(mn2, dot3(u, V2[k]));
      }
      return mn2 - mx1;
    };
    constexpr int NONE = 1 << 20;
    // Near-equal axes (parallel faces of the two feet, an edge axis equal to a face normal)
    // differ only by rounding, so the choice among them is made with a tolerance both the fp32
    // kernel and the fp64 oracle resolve the same way: the lowest-index face within TIE of the
    // best face, and an edge pair only when it beats that face by more than TIE.
    constexpr float TIE = Md::HULL_SAT_TIE;
    // face axes a = side * NF + f (u = FA[f] or FB[f]), NFL per lane kept in registers
    constexpr int NFL = (2 * NF + TEAM - 1) / TEAM;
    float fs[NFL], fmx = -1e30f, anysep = 0.0f;
#pragma unroll
    for (int k = 0; k < NFL; k++) {
      const int a = lane + TEAM * k;
      fs[k] = -1e30f;
      if (a < 2 * NF) {
        const int o = a < NF ? FA + 3 * a : FB + 3 * (a - NF);
        const float u[3] = {L[o], L[o + 1], L[o + 2]};
        const float sp = sep_of(u);
        anysep += sp > 0.0f ? 1.0f : 0.0f;
        fs[k] = sp;
      }
      fmx = fmaxf(fmx, fs[k]);
    }
    if (tsum(anysep) > 0.0f) return;
    const float ftop = tmaxf(fmx);
    int mine = NONE;
#pragma unroll
    for (int k = NFL - 1; k >= 0; k--)
      if (fs[k] >= ftop - TIE) mine = lane + TEAM * k;
    const int fbest = tmini(mine);
    float myf = fs[0];
#pragma unroll
    for (int k = 1; k < NFL; k++) myf = fbest / TEAM == k ? fs[k] : myf;
    float best = __shfl(myf, fbest % TEAM, TEAM);
    int btype = fbest / NF, bi = fbest - btype * NF, bj = 0;
    float u_best[3];
    {
      const int o = btype == 0 ? FA + 3 * bi : FB + 3 * bi;
      for (int q = 0; q < 3; q++) u_best[q] = L[o + q];
    }
    // edge-pair axes q = e1 * NE + e2 (lane: e2 = lane + 16 k), only pairs whose Gauss-map arcs
    // cross (a face of the Minkowski difference; the others are never the deepest axis but can
    // tie with it and would place the contact at a clamped segment end); any separation ends
    // the test
    constexpr int NEL = (NE + TEAM - 1) / TEAM;
    float EBr[NEL][3], Cr[NEL][3], Dr[NEL][3], DxC[NEL][3];
#pragma unroll
    for (int k = 0; k < NEL; k++) {
      const int e2 = lane + TEAM * k, e2c = e2 < NE ? e2 : 0;
      const int fc = HEF[e2c][0], fd = HEF[e2c][1];
      for (int q = 0; q < 3; q++) {
        EBr[k][q] = L[EB + 3 * e2c + q];
        Cr[k][q] = L[FB + 3 * fc + q];
        Dr[k][q] = L[FB + 3 * fd + q];
      }
      cross3(DxC[k], Dr[k], Cr[k]);
    }
    float esep = -1e30f, eu[3] = {0.0f, 0.0f, 1.0f};
    int eidx = NONE;
    for (int e1 = 0; e1 < NE; e1++) {
      const float ea[3] = {L[EA + 3 * e1], L[EA + 3 * e1 + 1], L[EA + 3 * e1 + 2]};
      const int fa = HEF[e1][0], fb = HEF[e1][1];
      const float A[3] = {L[FA + 3 * fa], L[FA + 3 * fa + 1], L[FA + 3 * fa + 2]};
      const float B[3] = {L[FA + 3 * fb], L[FA + 3 * fb + 1], L[FA + 3 * fb + 2]};
      float BxA[3];
      cross3(BxA, B, A);
      float sepq = 0.0f;
#pragma unroll
      for (int k = 0; k < NEL; k++) {
        const int e2 = lane + TEAM * k;
        const float CBA = dot3(Cr[k], BxA), DBA = dot3(Dr[k], BxA), ADC = dot3(A, DxC[k]), BDC = dot3(B, DxC[k]);
        if (e2 < NE && CBA * DBA < 0.0f && ADC * BDC < 0.0f && CBA * BDC > 0.0f) {
          float u[3];
          cross3(u, ea, EBr[k]);
          const float un = sqrtf(dot3(u, u));
          if (!(un < 1e-6f * sqrtf(dot3(ea, ea)) * sqrtf(dot3(EBr[k], EBr[k])))) {
            u[0] /= un; u[1] /= un; u[2] /= un;
            if (dot3(u, cc) < 0.0f) { u[0] = -u[0]; u[1] = -u[1]; u[2] = -u[2]; }
            const float sp = sep_of(u);
            sepq += sp > 0.0f ? 1.0f : 0.0f;
            if (sp > esep) { esep = sp; eidx = e1 * NE + e2; eu[0] = u[0]; eu[1] = u[1]; eu[2] = u[2]; }
          }
        }
      }
      if (tsum(sepq) > 0.0f) return;
    }
    const float em = tmaxf(esep);
    const int ebest = tmini(esep == em ? eidx : NONE);
    float u_edge[3];
    for (int q = 0; q < 3; q++) u_edge[q] = __shfl(eu[q], (ebest % NE) % TEAM, TEAM);  // lane of e2
    if (ebest < NONE && em > best + TIE) {
      best = em;
      btype = 2;
      bi = ebest / NE;
      bj = ebest - bi * NE;
      for (int q = 0; q < 3; q++) u_best[q] = u_edge[q];
    }
    // the contact, uniform over the team (the single-lane code's tail)
    TSYNC();
    float fr[9];
    make_frame(fr, u_best);
    if (btype == 2) {
      float a0[3], a1[3], b0[3], b1[3];
      pick3<NH>(V1, HE[bi][0], a0);
      pick3<NH>(V1, HE[bi][1], a1);
      pick3<NH>(V2, HE[bj][0], b0);
      pick3<NH>(V2, HE[bj][1], b1);
      float d1[3], d2[3], r[3];
      for (int a = 0; a < 3; a++) { d1[a] = a1[a] - a0[a]; d2[a] = b1[a] - b0[a]; r[a] = a0[a] - b0[a]; }
      const float A = dot3(d1, d1), E = dot3(d2, d2), F = dot3(d2, r), C = dot3(d1, r), B = dot3(d1, d2);
      const float den = A * E - B * B;
      float sc = den > 1e-15f ? (B * F - C * E) / den : 0.0f;
      sc = fminf(fmaxf(sc, 0.0f), 1.0f);
      float tt = E > 1e-15f ? (B * sc + F) / E : 0.0f;
      if (tt < 0.0f) { tt = 0.0f; sc = A > 1e-15f ? -C / A : 0.0f; }
      else if (tt > 1.0f) { tt = 1.0f; sc = A > 1e-15f ? (B - C) / A : 0.0f; }
      sc = fminf(fmaxf(sc, 0.0f), 1.0f);
      float pos[3];
      for (int a = 0; a < 3; a++) pos[a] = 0.5f * (a0[a] + sc * d1[a] + b0[a] + tt * d2[a]);
      if (lane == 0) P1::store_contact(Ls, slot0, best, pos, fr);
      return;
    }
    // face contact, mjx's clipped manifold (oracle collide_convex_convex): the incident face (the
    // other hull's face most anti-parallel to the reference normal, the first among equal ones)
    // clipped by the reference face's side planes (Sutherland-Hodgman in the reference polygon's
    // order; every lane runs the same clip through the dead edge scratch), the clipped points below
    // the reference plane, 4 of them by _manifold_points, each midway to the reference plane
    const bool ref1 = btype == 0;
    const float* Rr = ref1 ? R1 : R2;
    const float* Ri = ref1 ? R2 : R1;
    const float* pr = ref1 ? p1 : p2;
    float fn[3];
    mulmv3(fn, Rr, HN[bi]);
    const float off = Md::hull_face_offset_d()[bi] + dot3(fn, pr);
    int finc = 0;
    float dmin = 1e30f;
    for (int f = 0; f < NF; f++) {
      float ni[3];
      mulmv3(ni, Ri, HN[f]);
      const float dd = dot3(ni, fn);
      finc = dd < dmin ? f : finc;
      dmin = fminf(dmin, dd);
    }
    constexpr int MFV = Md::HULL_MAXFV, CLIPMAX = 2 * MFV;
    constexpr int PA = EA, PB = EA + 3 * CLIPMAX;
    static_assert(PB + 3 * CLIPMAX <= FA, "clip scratch must fit in the edge storage");
    const int(*FV)[MFV] = Md::hull_face_vert_d();
    const int* FNV = Md::hull_face_nv_d();
    auto vtx = [&](bool h1, int k, float* out) {
      float o1[3], o2[3];
      pick3<NH>(V1, k, o1);
      pick3<NH>(V2, k, o2);
      for (int q = 0; q < 3; q++) out[q] = h1 ? o1[q] : o2[q];
    };
    int np = FNV[finc];
    for (int i = 0; i < np; i++) {
      float v[3];
      vtx(!ref1, FV[finc][i], v);
      for (int q = 0; q < 3; q++) L[PA + 3 * i + q] = v[q];
    }
    int src = PA, dst = PB;
    const int nr = FNV[bi];
    for (int i = 0; i < nr && np > 0; i++) {
      float a[3], b[3], ab[3], sd[3];
      vtx(ref1, FV[bi][i], a);
      vtx(ref1, FV[bi][i + 1 < nr ? i + 1 : 0], b);
      for (int q = 0; q < 3; q++) ab[q] = b[q] - a[q];
      cross3(sd, ab, fn);  // outward side normal of the reference polygon's edge a -> b
      int nt = 0;
      for (int j = 0; j < np; j++) {
        const int jn = j + 1 < np ? j + 1 : 0;
        const float P[3] = {L[src + 3 * j], L[src + 3 * j + 1], L[src + 3 * j + 2]};
        const float Q[3] = {L[src + 3 * jn], L[src + 3 * jn + 1], L[src + 3 * jn + 2]};
        const float dp = sd[0] * (P[0] - a[0]) + sd[1] * (P[1] - a[1]) + sd[2] * (P[2] - a[2]);
        const float dq = sd[0] * (Q[0] - a[0]) + sd[1] * (Q[1] - a[1]) + sd[2] * (Q[2] - a[2]);
        if (dp <= 0.0f && nt < CLIPMAX) {
          for (int q = 0; q < 3; q++) L[dst + 3 * nt + q] = P[q];
          nt++;
        }
        if ((dp <= 0.0f) != (dq <= 0.0f) && nt < CLIPMAX) {
          const float tt = dp / (dp - dq);
          for (int q = 0; q < 3; q++) L[dst + 3 * nt + q] = P[q] + tt * (Q[q] - P[q]);
          nt++;
        }
      }
      TSYNC();
      np = nt;
      const int sw = src;
      src = dst;
      dst = sw;
    }
    float poly[CLIPMAX][3], depth[CLIPMAX];
    bool mask[CLIPMAX], any = false;
#pragma unroll
    for (int k = 0; k < CLIPMAX; k++) {
      const bool ok = k < np;
      for (int q = 0; q < 3; q++) poly[k][q] = ok ? L[src + 3 * k + q] : 0.0f;
      depth[k] = off - dot3(fn, poly[k]);
      mask[k] = ok && depth[k] > 0.0f;
      any = any || mask[k];
    }
    if (!any) return;
    int idx[4];
    manifold_points<CLIPMAX>(poly, mask, fn, idx);
    if (lane < 4) {
      const int c = lane;
      bool unique = true;
      for (int e = 0; e < 4; e++) unique = unique && !(e < c && idx[e] == idx[c]);
      const float dist = unique ? -pick1<CLIPMAX>(depth, idx[c]) : 1.0f;
      float v[3], pos[3];
      pick3<CLIPMAX>(poly, idx[c], v);
      for (int a = 0; a < 3; a++) pos[a] = v[a] - 0.5f * dist * fn[a];
      P1::store_contact(Ls, slot0 + c, dist, pos, fr);
    }
  }

  // out of line (frames recomputed) so the rare hull/hull SAT does not share the hot path's
  // code layout and registers
  static DNI void collide_hulls_rare(LP L, int lane) {
    constexpr int p = Md::FOOT_PAIR < 0 ? 0 : Md::FOOT_PAIR;
    const int s1 = cgeom_slot<Md>(Md::pair_geom1[p]), s2 = cgeom_slot<Md>(Md::pair_geom2[p]);
    S1 Ls{L};
    float p1[3], R1[9], p2[3], R2[9], t[3], c1[3], c2[3];
    P1::geom_frame(Ls, s1, p1, R1);
    P1::geom_frame(Ls, s2, p2, R2);
    const float hc[3] = {Md::hull_center[0], Md::hull_center[1], Md::hull_center[2]};
    mulmv3(t, R1, hc);
    for (int a = 0; a < 3; a++) c1[a] = p1[a] + t[a];
    mulmv3(t, R2, hc);
    for (int a = 0; a < 3; a++) c2[a] = p2[a] + t[a];
    const float cc[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
    collide_hulls_team(L, lane, 4 * p, p1, R1, p2, R2, cc);
  }

  static DK void collision(LP L, int lane, const float* hf) {
    STAGE_T0();
    if constexpr (Md::FLOOR_TYPE == 1) collide_hfield(L, lane, hf);
    else collide_planes(L, lane);
    STAGE_MARK(26);
    if (Md::FOOT_PAIR >= 0) {
      constexpr int p = Md::FOOT_PAIR;
      const int s1 = cgeom_slot<Md>(Md::pair_geom1[p]), s2 = cgeom_slot<Md>(Md::pair_geom2[p]);
      S1 Ls{L};
      // bounding-sphere reject (the common case) is uniform over the team
      float p1[3], R1[9], p2[3], R2[9], t[3];
      P1::geom_frame(Ls, s1, p1, R1);
      P1::geom_frame(Ls, s2, p2, R2);
      float c1[3], c2[3];
      const float hc[3] = {Md::hull_center[0], Md::hull_center[1], Md::hull_center[2]};
      mulmv3(t, R1, hc);
      for (int a = 0; a < 3; a++) c1[a] = p1[a] + t[a];
      mulmv3(t, R2, hc);
      for (int a = 0; a < 3; a++) c2[a] = p2[a] + t[a];
      const float cc[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
      if (dot3(cc, cc) > 4.0f * Md::hull_radius * Md::hull_radius || boxes_separated(p1, R1, p2, R2)) {
        if (lane < 4) {
          const float nofr[9] = {0, 0, 1, 0, 1, 0, -1, 0, 0};
          const float zero[3] = {L[Ly::COM], L[Ly::COM + 1], L[Ly::COM + 2]};
          P1::store_contact(Ls, 4 * p + lane, 1.0f, zero, nofr);
        }
      } else {
        TSYNC();
#ifdef DUCK_STAGE_PROF
        if (lane == 0) STAGE_ADD(27, 1ull);  // how often the SAT path runs
#endif
#ifndef DUCK_DIAG_NO_RARE_CALLS
        collide_hulls_rare(L, lane);  // rare: the boxes overlap
#endif
      }
    }
    TSYNC();
  }

  // ---------------- constraint rows ----------------
  static DK void make_rows(LP L, int lane) {
    if (lane < NFRIC) {
      const int r = lane, i = fric_dof(r);
      L[Ly::RD + r] = tf(Md::B_FRIC + 3 * r + 1);
      L[Ly::AREF + r] = -tf(Md::B_FRIC + 3 * r + 2) * L[Ly::QVEL + i];
    }
    team_for<NLIM>(lane, [&](int r) {
      const int o = Md::B_LIM + LIMW * r;
      const int i = lim_dof(r), qa = lim_qadr(r);
      const float q = L[Ly::QPOS + qa];
      const float dlo = q - tf(o + 2), dhi = tf(o + 3) - q;
      const float pos = fminf(dlo, dhi) - tf(o + 4);
      const float sgn = dlo < dhi ? 1.0f : -1.0f;
      const float k = tf(o + 5), b = tf(o + 6);
      const float si[5] = {tf(o + 8), tf(o + 9), tf(o + 10), tf(o + 11), tf(o + 12)};
      const float imp = imp_of(si, pos);
      const float R = fmaxf(tf(o + 7) * (1.0f - imp) * frcp(imp), 1e-15f);
      const bool active = pos < 0.0f;
      L[Ly::RD + R_LIM + r] = active ? frcp(R) : 0.0f;
      L[Ly::AREF + R_LIM + r] = active ? (-b * sgn * L[Ly::QVEL + i] - k * imp * pos) : 0.0f;
      L[Ly::LSGN + r] = sgn;
    });
    if (lane < NCON) {
      const int slot = lane, p = slot >> 2, o = Md::B_PAIR + PAIRW * p;
      float SL[6], SR[6];
      for (int k = 0; k < 6; k++) { SL[k] = L[Ly::CVEL + 6 * Md::LFOOT_BODY + k]; SR[k] = L[Ly::CVEL + 6 * Md::RFOOT_BODY + k]; }
      const float pos = L[Ly::CDIST + slot] - tf(o + 4);
      const bool active = pos < 0.0f;
      const float k = tf(o + 5), b = tf(o + 6);
      const float si[5] = {tf(o + 8), tf(o + 9), tf(o + 10), tf(o + 11), tf(o + 12)};
      const float imp = imp_of(si, pos);
      const float R = fmaxf(tf(o + 3) * (1.0f - imp) * frcp(imp), 1e-15f);
      float vel[4];
      contact_jx(L, p, slot, SL, SR, vel);
      for (int e = 0; e < 4; e++) {
        const int row = R_CON + 4 * slot + e;
        L[Ly::RD + row] = active ? frcp(R) : 0.0f;
        L[Ly::AREF + row] = active ? (-b * vel[e] - k * imp * pos) : 0.0f;
      }
    }
    TSYNC();
  }

  // J.x of one contact slot (4 pyramid edges) for body spatial motions SL/SR (runtime pair)
  static DK void contact_jx(LP L, int p, int slot, const float* SL, const float* SR, float* out4) {
    // contractions within expressions only: this function's statements are inlined into the fused warm
    // start of step_kernel and into the split halves of the latency kernels, where the backend formed
    // different FMAs across them (the flat scenes' kernels then agreed only to fp32 rounding;
    // tools/fpc_bisect.py located it, profiles/r05_lat_bitcmp.txt). With it the kernels agree bit for bit.
#pragma clang fp contract(on)
    const int o = Md::B_PAIR + PAIRW * p;
    const int s1 = ti(o), s2 = ti(o + 1);
    const float mu = tf(o + 2);
    const float r[3] = {L[Ly::CR + 3 * slot], L[Ly::CR + 3 * slot + 1], L[Ly::CR + 3 * slot + 2]};
    float v[3] = {0.0f, 0.0f, 0.0f}, t[3];
    if (s2 != 0) { P1::contact_vel(s2 == 1 ? SL : SR, r, t); v[0] += t[0]; v[1] += t[1]; v[2] += t[2]; }
    if (s1 != 0) { P1::contact_vel(s1 == 1 ? SL : SR, r, t); v[0] -= t[0]; v[1] -= t[1]; v[2] -= t[2]; }
    float jr[3];
    for (int q = 0; q < 3; q++)
      jr[q] = L[Ly::CFR + 9 * slot + 3 * q] * v[0] + L[Ly::CFR + 9 * slot + 3 * q + 1] * v[1] +
              L[Ly::CFR + 9 * slot + 3 * q + 2] * v[2];
    out4[0] = jr[0] + mu * jr[1];
    out4[1] = jr[0] - mu * jr[1];
    out4[2] = jr[0] + mu * jr[2];
    out4[3] = jr[0] - mu * jr[2];
  }

  // ---------------- Newton solver pieces ----------------
  static DK constexpr int kidx(int q, int k) {
    // packed upper-triangular index of (min(q,k), max(q,k)) in a 6x6 symmetric block
    return q <= k ? (q * 6 - (q * (q - 1)) / 2 + (k - q)) : (k * 6 - (k * (k - 1)) / 2 + (q - k));
  }

  // a line-search point: alpha, the team-summed linear and quadratic coefficients, the slope and
  // curvature, and this lane's un-summed constant coefficient (the cost is only needed for the final
  // bracket ends, so its team sum is deferred to them)
  struct Pt { float alpha, q0p, q1, q2, d0, d1; };

  // ---- fused solver passes ----
  // foot spatial motions only: component lane of X (lanes 0-11: left foot 0-5, right foot 6-11)
  // into so, of X2 (if >= 0) into so2; consumers take them by DPP row broadcasts (no LDS round trip)
  static DK void spatial2(LP L, int lane, int X, int X2, float& so, float& so2) {
    so = 0.0f;
    so2 = 0.0f;
    if (lane < 12) {
      // the feet's dof chains are compile-time (Md::chain): at each chain position the lane only
      // selects the left or right foot's dof, so no index words are loaded and the products of
      // all positions issue back to back. The lane is made opaque here: otherwise those per-lane
      // selects are hoisted out of the substep loop and held in registers for the whole kernel
      // (+15 AGPRs, -1.6 % same-box)
      int lo = lane;
      asm volatile("" : "+v"(lo));
      const bool left = lo < 6;
      const int k = left ? lo : lo - 6;
      float s = 0.0f, s2 = 0.0f;
#pragma unroll
      for (int c = 0; c < Md::MAXCHAIN; c++) {
        const int iL = Md::chain[Md::LFOOT_BODY][c], iR = Md::chain[Md::RFOOT_BODY][c];
        if (iL < 0 && iR < 0) continue;
        const bool ok = left ? iL >= 0 : iR >= 0;
        const int ic = left ? (iL >= 0 ? iL : 0) : (iR >= 0 ? iR : 0);
        if (FREE0 && iL == iR && iL >= 0 && iL < 3) {  // cdof = e_{3+i}: only lane k = 3 + i adds x
          const float x = L[X + iL];
          s += k == 3 + iL ? x : 0.0f;
          if (X2 >= 0) {
            const float x2 = L[X2 + iL];
            s2 += k == 3 + iL ? x2 : 0.0f;
          }
          continue;
        }
        const float cv = L[Ly::CDOF + 6 * ic + k];
        const float cd = ok ? cv : 0.0f;
        s += cd * L[X + ic];
        if (X2 >= 0) s2 += cd * L[X2 + ic];
      }
      so = s;
      so2 = s2;
    }
  }

  // SL[k] = component k of the left foot's motion (lane k), SR[k] the right foot's (lane 6 + k)
  static DK void sp_bcast(float v, float* SL, float* SR) {
    SL[0] = bc<0>(v); SL[1] = bc<1>(v); SL[2] = bc<2>(v); SL[3] = bc<3>(v); SL[4] = bc<4>(v); SL[5] = bc<5>(v);
    SR[0] = bc<6>(v); SR[1] = bc<7>(v); SR[2] = bc<8>(v); SR[3] = bc<9>(v); SR[4] = bc<10>(v); SR[5] = bc<11>(v);
  }

  static DK float fric_cost(float D, float x, float f) {
    const float rf = f * frcp(D);
    // the three pieces computed unconditionally and selected (nested ?: on expressions compiles to
    // branches)
    const float lo = -f * x - 0.5f * rf * f, hi = f * x - 0.5f * rf * f, qd = 0.5f * D * x * x;
    const float r = x >= rf ? hi : qd;
    return x <= -rf ? lo : r;
  }

  // the lane's constraint rows for the line search: its friction row, limit rows, and the
  // 4 edges of its contact slot (the same rows the lane computes J.x for)
  static constexpr int NLR = (NLIM + TEAM - 1) / TEAM;
  // Along the search line every row's cost is a fixed quadratic in alpha inside each zone,
  // so its coefficients are formed once: a one-sided row contributes (Q0, Q1, Q2) where
  // ja + alpha v < 0; the friction row (Huber) its quadratic zone or a linear piece.
  struct Rows2 {
    float fja, fv, frf, flin0, ffja, ffv, fQ0, fQ1, fQ2;  // friction row (zeros off the friction lanes)
    float ja[NLR + 4], v[NLR + 4], Q0[NLR + 4], Q1[NLR + 4], Q2[NLR + 4];  // limit rows, then contact edges
  };
  static DK void set_fric(Rows2& R, float D, float ja, float v, float f) {
    const float rf = f * frcp(D);
    R.fja = ja; R.fv = v; R.frf = rf;
    R.flin0 = -0.5f * rf * f; R.ffja = f * ja; R.ffv = f * v;
    R.fQ0 = 0.5f * D * ja * ja; R.fQ1 = D * v * ja; R.fQ2 = 0.5f * D * v * v;
  }
  static DK void set_row(Rows2& R, int k, float D, float ja, float v) {
    R.ja[k] = ja; R.v[k] = v;
    R.Q0[k] = 0.5f * D * ja * ja; R.Q1[k] = D * v * ja; R.Q2[k] = 0.5f * D * v * v;
  }

  // partial quadratic coefficients of this lane's rows at alpha (branchless)
  static DK void quad2(const Rows2& R, float alpha, float& q0, float& q1, float& q2) {
    {
      const float x = R.fja + alpha * R.fv;
      const bool lo = x <= -R.frf, hi = x >= R.frf, quad = !(lo || hi);
      const float sg = lo ? -1.0f : 1.0f;
      q0 += quad ? R.fQ0 : R.flin0 + sg * R.ffja;
      q1 += quad ? R.fQ1 : sg * R.ffv;
      q2 += quad ? R.fQ2 : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < NLR + 4; k++) {
      const float on = (R.ja[k] + alpha * R.v[k] < 0.0f) ? 1.0f : 0.0f;
      q0 = fmaf(on, R.Q0[k], q0);
      q1 = fmaf(on, R.Q1[k], q1);
      q2 = fmaf(on, R.Q2[k], q2);
    }
  }

  // mjx solver.solve: warm-start choice, then Md::iterations Newton steps (the Open Duck scenes
  // use 1; a model compiled with more iterates to the MJX stopping rule on the cost improvement)
  // Mc: M as full symmetric columns in registers for every M.x of the solver
  static DK void solve(LP L, int lane, float* scratch, int stride, const float (*Mc)[NV]) {
    STAGE_T0();
    const float g0 = warm_start(L, lane, Mc);
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 21
    (void)warm_start(L, lane, Mc);
#endif
    newton(L, lane, scratch, stride, Mc, g0);
  }
  // latency mode: the warm start's products that need only qacc_warmstart (its feet motions, M and J
  // products, constraint costs) run while wave 3 solves for qacc_smooth; then those of qacc_smooth
  // and the choice. The same operations in the same order as warm_start's fused pass: same values.
  // (a0 needs only qacc_warmstart and M: it runs before the rows are there; a1 the rows' costs)
  static DK void warm_start_a0(LP L, int lane, const float (*Mc)[NV], float* SL, float* SR) {
    float sw, ss;
    spatial2(L, lane, Ly::WARM, -1, sw, ss);
    {
      float xw[NC];
      lane_vec(L, lane, Ly::WARM, xw);
      mul_cols(L, lane, Mc, xw, Ly::MA);  // (MA is read after the next team sync)
    }
    sp_bcast(sw, SL, SR);
  }
  static DK void warm_start_a1(LP L, int lane, const float* SL, const float* SR, float& cwp) {
    cwp = 0.0f;
    {
      const bool fr = lane < NFRIC;
      const int r = fr ? lane : 0, i = fric_dof(r);
      const float D = L[Ly::RD + r], f = L[Ly::DFRIC + i], ar = L[Ly::AREF + r];
      const float jw = L[Ly::WARM + i] - ar;
      cwp += fr ? fric_cost(D, jw, f) : 0.0f;
      L[fr ? Ly::JA + r : TL::SINK + lane] = jw;
    }
    team_for<NLIM>(lane, [&](int r) {
      const int i = lim_dof(r), row = R_LIM + r;
      const float D = L[Ly::RD + row], sg = L[Ly::LSGN + r], ar = L[Ly::AREF + row];
      const float jw = sg * L[Ly::WARM + i] - ar;
      cwp += jw < 0.0f ? 0.5f * D * jw * jw : 0.0f;
      L[Ly::JA + row] = jw;
    });
    if (lane < NCON) {
      float vw[4];
      contact_jx(L, lane >> 2, lane, SL, SR, vw);
      for (int e = 0; e < 4; e++) {
        const int row = R_CON + 4 * lane + e;
        const float D = L[Ly::RD + row], ar = L[Ly::AREF + row];
        const float jw = vw[e] - ar;
        cwp += jw < 0.0f ? 0.5f * D * jw * jw : 0.0f;
        L[Ly::JA + row] = jw;
      }
    }
  }
  static DK float warm_start_b(LP L, int lane, float cwp, bool& warm) {
    float ss, s2;
    spatial2(L, lane, Ly::QSM, -1, ss, s2);
    TSYNC();
    float SL2[6], SR2[6];
    sp_bcast(ss, SL2, SR2);
    float csp = 0.0f, gwp = 0.0f;
    {
      const bool fr = lane < NFRIC;
      const int r = fr ? lane : 0, i = fric_dof(r);
      const float D = L[Ly::RD + r], f = L[Ly::DFRIC + i], ar = L[Ly::AREF + r];
      const float js = L[Ly::QSM + i] - ar;
      csp += fr ? fric_cost(D, js, f) : 0.0f;
      L[fr ? Ly::JV + r : TL::SINK + TEAM + lane] = js;
    }
    team_for<NLIM>(lane, [&](int r) {
      const int i = lim_dof(r), row = R_LIM + r;
      const float D = L[Ly::RD + row], sg = L[Ly::LSGN + r], ar = L[Ly::AREF + row];
      const float js = sg * L[Ly::QSM + i] - ar;
      csp += js < 0.0f ? 0.5f * D * js * js : 0.0f;
      L[Ly::JV + row] = js;
    });
    if (lane < NCON) {
      float vs[4];
      contact_jx(L, lane >> 2, lane, SL2, SR2, vs);
      for (int e = 0; e < 4; e++) {
        const int row = R_CON + 4 * lane + e;
        const float D = L[Ly::RD + row], ar = L[Ly::AREF + row];
        const float js = vs[e] - ar;
        csp += js < 0.0f ? 0.5f * D * js * js : 0.0f;
        L[Ly::JV + row] = js;
      }
    }
    team_for<NV>(lane, [&](int i) { gwp += 0.5f * (L[Ly::MA + i] - L[Ly::FSM + i]) * (L[Ly::WARM + i] - L[Ly::QSM + i]); });
    const float gw = tsum(gwp);
    const float cw = gw + tsum(cwp), cs = tsum(csp);
    float g0;
    warm = cw < cs;
    if (warm) {
      team_for<NV>(lane, [&](int i) { L[Ly::QACC + i] = L[Ly::WARM + i]; });
      g0 = gw;
    } else {
      team_for<NV>(lane, [&](int i) { L[Ly::QACC + i] = L[Ly::QSM + i]; L[Ly::MA + i] = L[Ly::FSM + i]; });
      team_for<NROW>(lane, [&](int r) { L[Ly::JA + r] = L[Ly::JV + r]; });
      g0 = 0.0f;
    }
    TSYNC();
    return g0;
  }
  // warm start vs smooth acceleration (mjx solver.solve's start): returns the Gauss cost at the start
  static DK float warm_start(LP L, int lane, const float (*Mc)[NV]) {
    STAGE_T0();
    // warm start vs smooth acceleration: J and M products of both in one pass
    // (M qacc_smooth = qfrc_smooth by definition: no product needed for the smooth start)
    float sw, ss;
    spatial2(L, lane, Ly::WARM, Ly::QSM, sw, ss);
    {
      float xw[NC];
      lane_vec(L, lane, Ly::WARM, xw);
      mul_cols(L, lane, Mc, xw, Ly::MA);
    }
    TSYNC();
    // the feet's spatial motions, broadcast with the full team active (before any lane region)
    float SL[6], SR[6], SL2[6], SR2[6];
    sp_bcast(sw, SL, SR);
    sp_bcast(ss, SL2, SR2);
    STAGE_MARK(25);
    float cwp = 0.0f, csp = 0.0f, gwp = 0.0f;
    {
      // branchless (no lane-divergent region: see TL::SINK)
      const bool fr = lane < NFRIC;
      const int r = fr ? lane : 0, i = fric_dof(r);
      const float D = L[Ly::RD + r], f = L[Ly::DFRIC + i], ar = L[Ly::AREF + r];
      const float jw = L[Ly::WARM + i] - ar, js = L[Ly::QSM + i] - ar;
      cwp += fr ? fric_cost(D, jw, f) : 0.0f;
      csp += fr ? fric_cost(D, js, f) : 0.0f;
      L[fr ? Ly::JA + r : TL::SINK + lane] = jw;
      L[fr ? Ly::JV + r : TL::SINK + TEAM + lane] = js;
    }
    team_for<NLIM>(lane, [&](int r) {
      const int i = lim_dof(r), row = R_LIM + r;
      const float D = L[Ly::RD + row], sg = L[Ly::LSGN + r], ar = L[Ly::AREF + row];
      const float jw = sg * L[Ly::WARM + i] - ar, js = sg * L[Ly::QSM + i] - ar;
      cwp += jw < 0.0f ? 0.5f * D * jw * jw : 0.0f;
      csp += js < 0.0f ? 0.5f * D * js * js : 0.0f;
      L[Ly::JA + row] = jw;
      L[Ly::JV + row] = js;
    });
    if (lane < NCON) {
      float vw[4], vs[4];
      contact_jx(L, lane >> 2, lane, SL, SR, vw);
      contact_jx(L, lane >> 2, lane, SL2, SR2, vs);
      for (int e = 0; e < 4; e++) {
        const int row = R_CON + 4 * lane + e;
        const float D = L[Ly::RD + row], ar = L[Ly::AREF + row];
        const float jw = vw[e] - ar, js = vs[e] - ar;
        cwp += jw < 0.0f ? 0.5f * D * jw * jw : 0.0f;
        csp += js < 0.0f ? 0.5f * D * js * js : 0.0f;
        L[Ly::JA + row] = jw;
        L[Ly::JV + row] = js;
      }
    }
    team_for<NV>(lane, [&](int i) { gwp += 0.5f * (L[Ly::MA + i] - L[Ly::FSM + i]) * (L[Ly::WARM + i] - L[Ly::QSM + i]); });
    const float gw = tsum(gwp);
    const float cw = gw + tsum(cwp), cs = tsum(csp);
    float g0;
    if (cw < cs) {
      team_for<NV>(lane, [&](int i) { L[Ly::QACC + i] = L[Ly::WARM + i]; });
      g0 = gw;
    } else {
      team_for<NV>(lane, [&](int i) { L[Ly::QACC + i] = L[Ly::QSM + i]; L[Ly::MA + i] = L[Ly::FSM + i]; });
      team_for<NROW>(lane, [&](int r) { L[Ly::JA + r] = L[Ly::JV + r]; });
      g0 = 0.0f;  // gauss(qacc_smooth) = 0.5 (M qs - f).(qs - qs) = 0
    }
    TSYNC();
    STAGE_MARK(9);
    return g0;
  }
  // Md::iterations Newton steps from the start in QACC / MA / JA (Gauss cost g0 there)
  // pre_dir (latency mode): the first direction is already in TL::XDIR (wave 3's, from the same inputs);
  // used when every team of the wave has one, else the wave computes it (the same values for those teams)
  static DK void newton(LP L, int lane, float* scratch, int stride, const float (*Mc)[NV], float g0,
                        bool pre_dir = false) {
    STAGE_T0();
    (void)scratch;
    (void)stride;
    for (int newton_it = 0;;) {
    bool sparse_ok;
    if (LAT && newton_it == 0 && __ballot(!pre_dir) == 0ull) {
      team_for<NV>(lane, [&](int i) { L[Ly::SRCH + i] = L[TL::XDIR + i]; });
      TSYNC();
      sparse_ok = true;
    } else {
      sparse_ok = newton_fused<false>(L, lane, Mc);
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 22
      sparse_ok = newton_fused<false>(L, lane, Mc);
#endif
    }
    STAGE_MARK(10);
    if (sparse_ok) {
      STAGE_MARK(11);
    } else {
      TSYNC();
#ifdef DUCK_STAGE_PROF
      if (lane == 0) STAGE_ADD(23, 1ull);  // dense Newton fallbacks
#endif
#ifndef DUCK_DIAG_NO_RARE_CALLS
      newton_dense(L, lane);  // rare: foot/foot contact rows active (dense H)
#endif
      TSYNC();
    }
    // J.search and M.search in one pass; rows go straight to registers
    float sv, sv2;
    spatial2(L, lane, Ly::SRCH, -1, sv, sv2);
    {
      float xs[NC];
      lane_vec(L, lane, Ly::SRCH, xs);
      mul_cols(L, lane, Mc, xs, Ly::GRAD);
    }
    TSYNC();
    Rows2 R;
    {
      const bool fr = lane < NFRIC;
      const int r = fr ? lane : 0, i = fric_dof(r);
      const float D = L[Ly::RD + r], ja = L[Ly::JA + r], v = L[Ly::SRCH + i], f = L[Ly::DFRIC + i];
      set_fric(R, fr ? D : 1.0f, fr ? ja : 0.0f, fr ? v : 0.0f, fr ? f : 0.0f);
    }
#pragma unroll
    for (int m = 0; m < NLR; m++) {
      const int r = lane + TEAM * m;
      const bool ok = r < NLIM;
      const int rc = ok ? r : 0, i = lim_dof(rc), row = R_LIM + rc;
      const float D = L[Ly::RD + row], ja = L[Ly::JA + row], v = L[Ly::LSGN + rc] * L[Ly::SRCH + i];
      set_row(R, m, ok ? D : 0.0f, ok ? ja : 0.0f, ok ? v : 0.0f);
    }
    {
      float SL[6], SR[6], v[4];
      const int slot = lane < NCON ? lane : 0;
      sp_bcast(sv, SL, SR);
      contact_jx(L, slot >> 2, slot, SL, SR, v);
      for (int e = 0; e < 4; e++) {
        const int row = R_CON + 4 * slot + e;
        const bool ok = lane < NCON;
        const float D = L[Ly::RD + row], ja = L[Ly::JA + row];
        set_row(R, NLR + e, ok ? D : 0.0f, ok ? ja : 0.0f, ok ? v[e] : 0.0f);
      }
    }
    float sn = 0.0f, sMa = 0.0f, sf = 0.0f, sMv = 0.0f;
#ifdef DUCK_LS_DUMP
    {
      const unsigned long long ex = __builtin_amdgcn_read_exec();
      L[TL::KC + 88 + lane] = __int_as_float((int)(ex & 0xffffffffull));
      L[TL::KC + 104 + lane] = __int_as_float((int)(ex >> 32));
      L[TL::KC + 120 + lane] = L[Ly::SRCH + lane];
    }
#endif
    team_for<NV>(lane, [&](int i) {
      const float sv = L[Ly::SRCH + i];
      sn += sv * sv;
      sMa += sv * L[Ly::MA + i];
      sf += sv * L[Ly::FSM + i];
      sMv += sv * L[Ly::GRAD + i];
    });
#ifdef DUCK_LS_DUMP
    L[TL::KC + 56 + lane] = (float)lane;
    L[TL::KC + 72 + lane] = sn;
#endif
    sn = tsum(sn); sMa = tsum(sMa); sf = tsum(sf); sMv = tsum(sMv);
    STAGE_MARK(12);
    const float gtol = Md::tolerance * Md::ls_tolerance * sqrtf(sn) * Md::meaninertia * (float)(NV > 1 ? NV : 1);
    const float G0 = g0, G1 = sMa - sf, G2 = 0.5f * sMv;
    auto mk = [&](float alpha, float q0, float q1, float q2) {
      q1 = tsum(q1) + G1; q2 = tsum(q2) + G2;
      Pt p;
      p.alpha = alpha;
      p.q0p = q0;
      p.q1 = q1;
      p.q2 = q2;
      p.d0 = 2.0f * alpha * q2 + q1;
      p.d1 = 2.0f * q2;
      return p;
    };
    auto cost = [&](const Pt& p) { return p.alpha * p.alpha * p.q2 + p.alpha * p.q1 + (tsum(p.q0p) + G0); };
    Pt p0;
    {
      float q0 = 0, q1 = 0, q2 = 0;
      quad2(R, 0.0f, q0, q1, q2);
#ifdef DUCK_LS_DUMP
      // debug builds: the line search's inputs, into the (dead) KC scratch of the env slice
      L[TL::KC + 8 + 3 * lane] = q0; L[TL::KC + 9 + 3 * lane] = q1; L[TL::KC + 10 + 3 * lane] = q2;
      if (lane == 0) { L[TL::KC] = G0; L[TL::KC + 1] = G1; L[TL::KC + 2] = G2; L[TL::KC + 3] = gtol; L[TL::KC + 4] = sn; }
#endif
      p0 = mk(0.0f, q0, q1, q2);
    }
    Pt lo;
    {
      // (as the loop's steps: alpha - d0 v_rcp(d1); written as a division this one, at alpha = 0, compiled
      // to the correctly rounded sequence with two MODE register writes)
      const float a1 = p0.alpha - p0.d0 * frcp(p0.d1);
      float q0 = 0, q1 = 0, q2 = 0;
      quad2(R, a1, q0, q1, q2);
      lo = mk(a1, q0, q1, q2);
    }
    Pt hi;
    if (lo.d0 < p0.d0) { hi = p0; } else { hi = lo; lo = p0; }
    bool swap = true;
    // fp32 termination floor: a bracket end whose slope is below 1e-6 of the starting slope is at the
    // minimum to fp32 resolution; MJX's gtol (tolerance * ls_tolerance * |search| ...) alone is far
    // below fp32 noise, so fp32 iterations would keep swapping on rounding
    const float gtol_ls = fmaxf(gtol, DUCK_LS_DFLOOR * fabsf(p0.d0));
#ifdef DUCK_LS_NOBREAK
    bool stop = false;
#pragma unroll
    for (int it = 0; it < Md::ls_iterations; it++) {
      bool done = stop || !swap;
      done = done || ((lo.d0 < 0.0f) && (lo.d0 > -gtol_ls));
      done = done || ((hi.d0 > 0.0f) && (hi.d0 < gtol_ls));
      stop = done;
#else
#ifdef DUCK_STAGE_PROF
    int its = 0;
#endif
    for (int it = 0; it < Md::ls_iterations; it++) {
      bool done = !swap;
      done = done || ((lo.d0 < 0.0f) && (lo.d0 > -gtol_ls));
      done = done || ((hi.d0 > 0.0f) && (hi.d0 < gtol_ls));
      if (done) break;
#ifdef DUCK_STAGE_PROF
      its = it + 1;
      if (threadIdx.x < 64 && (int)threadIdx.x == __ffsll((long long)__ballot(1)) - 1) STAGE_ADD(56, 1ull);
#endif
#endif
      const float al = lo.alpha - lo.d0 / lo.d1, ah = hi.alpha - hi.d0 / hi.d1, am = 0.5f * (lo.alpha + hi.alpha);
      float a0 = 0, a1 = 0, a2 = 0, b0 = 0, b1 = 0, b2 = 0, c0 = 0, c1 = 0, c2 = 0;
      quad2(R, al, a0, a1, a2);
      quad2(R, ah, b0, b1, b2);
      quad2(R, am, c0, c1, c2);
      const Pt lo_next = mk(al, a0, a1, a2), hi_next = mk(ah, b0, b1, b2), mid = mk(am, c0, c1, c2);
#ifdef DUCK_LS_NOBREAK
      const bool s1 = !done && ((lo.d0 > 0.0f) || (lo.d0 < lo_next.d0));
      if (s1) lo = lo_next;
      const bool s2 = !done && (mid.d0 < 0.0f) && (lo.d0 < mid.d0);
      if (s2) lo = mid;
      const bool s3 = !done && ((hi.d0 < 0.0f) || (hi.d0 > hi_next.d0));
      if (s3) hi = hi_next;
      const bool s4 = !done && (mid.d0 > 0.0f) && (hi.d0 > mid.d0);
      if (s4) hi = mid;
      swap = done ? swap : (s1 || s2 || s3 || s4);
#else
      const bool s1 = (lo.d0 > 0.0f) || (lo.d0 < lo_next.d0);
      if (s1) lo = lo_next;
      const bool s2 = (mid.d0 < 0.0f) && (lo.d0 < mid.d0);
      if (s2) lo = mid;
      const bool s3 = (hi.d0 < 0.0f) || (hi.d0 > hi_next.d0);
      if (s3) hi = hi_next;
      const bool s4 = (mid.d0 > 0.0f) && (hi.d0 > mid.d0);
      if (s4) hi = mid;
      swap = s1 || s2 || s3 || s4;
#endif
    }
#if defined(DUCK_STAGE_PROF) && !defined(DUCK_LS_NOBREAK)
    if (threadIdx.x < 64 && (lane & 15) == 0) { STAGE_ADD(57, (unsigned long long)its); STAGE_ADD(58, 1ull); }
#endif
    const float lo_cost = cost(lo), hi_cost = cost(hi), p0_cost = cost(p0);
    const bool improved = (lo_cost < p0_cost) || (hi_cost < p0_cost);
    const float alpha = lo_cost < hi_cost ? lo.alpha : hi.alpha;
    if (improved)
      team_for<NV>(lane, [&](int i) { L[Ly::QACC + i] += L[Ly::SRCH + i] * alpha; });
    TSYNC();
    STAGE_MARK(13);
    if constexpr (Md::iterations <= 1) {
      break;
    } else {
      // next Newton step from the new point (mjx solver.solve loop): M.qacc and J.qacc - aref move
      // along the search direction; stop on the iteration count or a cost improvement below
      // tolerance (the gradient-norm test is not repeated here: at that point the next step's
      // change is below fp32 resolution)
      if (++newton_it >= Md::iterations) break;
      const float a = improved ? alpha : 0.0f;
      const float cnew = improved ? (lo_cost < hi_cost ? lo_cost : hi_cost) : p0_cost;
      g0 = G0 + a * G1 + a * a * G2;  // gauss at the new point
      team_for<NV>(lane, [&](int i) { L[Ly::MA + i] += a * L[Ly::GRAD + i]; });  // GRAD = M.search
      if (lane < NFRIC) L[Ly::JA + lane] = R.fja + a * R.fv;
#pragma unroll
      for (int m = 0; m < NLR; m++) {
        const int r = lane + TEAM * m;
        if (r < NLIM) L[Ly::JA + R_LIM + r] = R.ja[m] + a * R.v[m];
      }
      if (lane < NCON)
        for (int e = 0; e < 4; e++) L[Ly::JA + R_CON + 4 * lane + e] = R.ja[NLR + e] + a * R.v[NLR + e];
      TSYNC();
      const float scale = 1.0f / (Md::meaninertia * (float)(NV > 1 ? NV : 1));
      if (scale * (p0_cost - cnew) < Md::tolerance) break;
    }
    }
  }

  // ---------------- sensors (last substep) ----------------
  static DK void sensors(LP L, int lane) {
    const float com[3] = {L[Ly::COM], L[Ly::COM + 1], L[Ly::COM + 2]};
    float cacc1[6];
    for (int k = 0; k < 6; k++) cacc1[k] = (k >= 3) ? -Md::gravity[k - 3] : 0.0f;
    for (int i = 0; i < 6; i++) {
      const float v = L[Ly::QVEL + i], a = L[Ly::QACC + i];
      for (int k = 0; k < 6; k++) {
        const float cdd = i >= 3 ? L[Ly::CDD1 + 6 * (i - 3) + k] : 0.0f;
        cacc1[k] += cdd * v + L[Ly::CDOF + 6 * i + k] * a;
      }
    }
    for (int s = lane; s < Md::NSENSOR; s += TEAM) {
      const int os = Md::B_SENS + 20 * s;
      const int typ = ti(os), site = ti(os + 1), adr = ti(os + 2), b = ti(os + 3);
      float R[9], sp[3], sR[9], t[3], SM[9];
      const float spos[3] = {tf(os + 4), tf(os + 5), tf(os + 6)};
      for (int k = 0; k < 9; k++) { R[k] = L[Ly::XMAT + 9 * b + k]; SM[k] = tf(os + 7 + k); }
      mulmv3(t, R, spos);
      for (int k = 0; k < 3; k++) sp[k] = L[Ly::XPOS + 3 * b + k] + t[k];
      mulmm3(sR, R, SM);
      const float off[3] = {sp[0] - com[0], sp[1] - com[1], sp[2] - com[2]};
      float ang[3] = {L[Ly::CVEL + 6 * b], L[Ly::CVEL + 6 * b + 1], L[Ly::CVEL + 6 * b + 2]}, lin[3];
      cross3(t, ang, off);
      for (int k = 0; k < 3; k++) lin[k] = L[Ly::CVEL + 6 * b + 3 + k] + t[k];
      float o[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (typ == 0) mulmtv3(o, sR, ang);
      else if (typ == 1) mulmtv3(o, sR, lin);
      else if (typ == 2) {
        float acc[3];
        cross3(t, cacc1, off);
        for (int k = 0; k < 3; k++) acc[k] = cacc1[3 + k] + t[k];
        cross3(t, ang, lin);
        for (int k = 0; k < 3; k++) acc[k] += t[k];
        mulmtv3(o, sR, acc);
      } else if (typ == 3) { o[0] = sR[2]; o[1] = sR[5]; o[2] = sR[8]; }
      else if (typ == 4) { o[0] = sR[0]; o[1] = sR[3]; o[2] = sR[6]; }
      else if (typ == 5) { o[0] = lin[0]; o[1] = lin[1]; o[2] = lin[2]; }
      else if (typ == 6) { o[0] = ang[0]; o[1] = ang[1]; o[2] = ang[2]; }
      else if (typ == 7) { o[0] = sp[0]; o[1] = sp[1]; o[2] = sp[2]; }
      else if (typ == 8) {
        const float bq[4] = {L[Ly::XQ + 4 * b], L[Ly::XQ + 4 * b + 1], L[Ly::XQ + 4 * b + 2], L[Ly::XQ + 4 * b + 3]};
        const float sq[4] = {tf(os + 16), tf(os + 17), tf(os + 18), tf(os + 19)};
        qmul(o, bq, sq);
        qnormalize(o);
      }
      const int dim = typ == 8 ? 4 : 3;
      for (int k = 0; k < dim; k++) L[Ly::SENS + adr + k] = o[k];
      if (typ == 0 && site == Md::IMU_SITE) { L[Ly::IMUR] = sR[6]; L[Ly::IMUR + 1] = sR[7]; L[Ly::IMUR + 2] = sR[8]; }
      if (typ == 7 && site == Md::LFOOT_SITE) L[Ly::FOOTZ] = sp[2];
      if (typ == 7 && site == Md::RFOOT_SITE) L[Ly::FOOTZ + 1] = sp[2];
    }
    if (lane < 2) {
      // (compile-time table entries selected by lane: indexed by lane, the tables were read from
      // global memory with an exposed load)
      constexpr int p0 = Md::PLANE_PAIR[0], p1 = Md::PLANE_PAIR[1];
      constexpr int s20 = cgeom_slot<Md>(Md::pair_geom2[p0]), s21 = cgeom_slot<Md>(Md::pair_geom2[p1]);
      const int p = lane == 0 ? p0 : p1, s2 = lane == 0 ? s20 : s21;
      float mn = 1e4f;
      for (int c = 0; c < 4; c++) mn = fminf(mn, L[Ly::CDIST + 4 * p + c]);
      L[Ly::OCON + s2 - 1] = mn < 0.0f ? 1.0f : 0.0f;
    }
    TSYNC();
  }

  // ---------------- semi-implicit Euler ----------------
  static DK void euler(LP L, int lane) {
    const float dt = Md::timestep;
    team_for<NV>(lane, [&](int i) {
      L[Ly::WARM + i] = L[Ly::QACC + i];
      L[Ly::QVEL + i] += dt * L[Ly::QACC + i];
    });
    TSYNC();
    if (lane == 0) {
      for (int k = 0; k < 3; k++) L[Ly::QPOS + k] += dt * L[Ly::QVEL + k];
      const float v[3] = {L[Ly::QVEL + 3], L[Ly::QVEL + 4], L[Ly::QVEL + 5]};
      const float nvv = sqrtf(dot3(v, v));
      float ax[3] = {1.0f, 0.0f, 0.0f};
      if (nvv > 1e-15f) { ax[0] = v[0] / nvv; ax[1] = v[1] / nvv; ax[2] = v[2] / nvv; }
      float s, c;
      __sincosf(0.5f * dt * nvv, &s, &c);
      const float qr[4] = {c, ax[0] * s, ax[1] * s, ax[2] * s};
      float q[4] = {L[Ly::QPOS + 3], L[Ly::QPOS + 4], L[Ly::QPOS + 5], L[Ly::QPOS + 6]};
      qmul(q, q, qr);
      qnormalize(q);
      for (int k = 0; k < 4; k++) L[Ly::QPOS + 3 + k] = q[k];
    }
    team_for<NJ, 1>(lane, [&](int j) {
      const int oj = Md::B_JREC + 9 * j;
      const bool jh = Md::B_JAFF && j >= Md::B_JN0;
      const int qa = jh ? j + Md::B_JQD : ti(oj + 2), da = jh ? j + Md::B_JDD : ti(oj + 1);
      L[Ly::QPOS + qa] += dt * L[Ly::QVEL + da];
    });
    TSYNC();
  }

  static DK void step(LP L, int lane, bool integrate, bool want_out, float* aux, int aux_stride, float* scratch,
                      int sstride, const float* hf) {
    STAGE_T0();
    kinematics(L, lane);
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 6
    kinematics(L, lane);
#endif
    STAGE_MARK(0);
    com_pos(L, lane);
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 7
    com_pos(L, lane);
#endif
    STAGE_MARK(1);
    rne(L, lane);
    STAGE_MARK(2);
    crb(L, lane);
    // DUCK_DOUBLE (measurement builds, tools/gpu_stage_double.sh, tools/gpu_stage_pmc.sh): one
    // idempotent stage runs twice, and the launch-time (and counter) difference to the normal build
    // is that stage's cost, unperturbed by markers: 1 crb, 2 collision, 3 make_rows, 4 smooth_acc,
    // 5 solve, 6 kinematics, 7 com_pos, 8 rne + smooth (height field: 11-20, tools/stage_pmc_summary.py)
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 1
    crb(L, lane);
#endif
    STAGE_MARK(3);
    smooth(L, lane);
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 8
    rne(L, lane);  // (smooth adds to rne's qfrc_smooth: the pair is idempotent, smooth alone is not)
    smooth(L, lane);
#endif
    STAGE_MARK(28);
    // collision and the constraint rows depend on the kinematics only: they run before the
    // smooth acceleration so that M is loaded into registers once for both solves
    collision(L, lane, hf);
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 2
    collision(L, lane, hf);
#endif
    STAGE_MARK(5);
    make_rows(L, lane);
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 3
    make_rows(L, lane);
#endif
    STAGE_MARK(6);
    {
      float Mc[NC][NV];
      load_cols(L, lane, Mc, false);
      STAGE_MARK(20);
      smooth_acc(L, lane, Mc);
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 4
      smooth_acc(L, lane, Mc);
#endif
      STAGE_MARK(4);
      solve(L, lane, scratch, sstride, Mc);
#if defined(DUCK_DOUBLE) && DUCK_DOUBLE == 5
      solve(L, lane, scratch, sstride, Mc);  // (reads qacc_warmstart / qacc_smooth, not qacc)
#endif
    }
    STAGE_MARK(7);
    if (want_out) {
      sensors(L, lane);
      if (aux) {
        S1 Ls{L};
        if (lane == 0) P1::write_aux(Ls, aux, aux_stride);
      }
    }
    if (integrate) {
      euler(L, lane);
    } else {
      team_for<NV>(lane, [&](int i) { L[Ly::WARM + i] = L[Ly::QACC + i]; });
      TSYNC();
    }
    STAGE_MARK(8);
  }

  // ---------------- latency mode: one substep over three waves (step_kernel_lat) ----------------
  // Cross-wave events are counters in LDS (one 16-B group each, after the slices): the producer
  // wave stores the number of the substep it finished (a workgroup-scope release: its LDS writes
  // complete first), a consumer spins on an acquire load until the count is reached. Counts only
  // grow within a launch, so no event is reset between substeps. A spin is bounded (~40 ms, far
  // beyond a substep) so that a broken schedule ends the launch instead of hanging the device;
  // g_lat_timeouts counts such exits (tests read it: it must stay 0).
  // EV_TIMEOUT is not an event: a wait that gave up sets it, and step_kernel_lat then raises the
  // handle's sticky device error word and writes NaN qpos for the workgroup's envs (duck_device_error)
  enum { EV_KIN = 0, EV_VEL = 1, EV_FSM = 2, EV_ROWS = 3, EV_EULER = 4, EV_M = 5, EV_QSM = 6, EV_WA = 7, EV_DIR = 8,
         EV_TIMEOUT = 9 };
  static_assert(EV_TIMEOUT < TL::NEV_G || !LAT, "event slots");
  // the paired kernel (LAT 2): waves 2w and 2w + 1 work env set w, whose events are its own group
  static DK lds_int* ev_ptr(int k) {
    extern __shared__ float lds_dyn[];
    const int g = LAT == 2 ? __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 7) : 0;
    return (lds_int*)(lds_dyn + TL::EV) + 4 * (k + TL::NEV_G * g);
  }
  static DK void ev_init(int tid) {
    extern __shared__ float lds_dyn[];
    if (tid < TL::NEV) ((lds_int*)(lds_dyn + TL::EV))[4 * tid] = 0;
  }
  static DK void ev_signal(int k, int v) {
    __hip_atomic_store(ev_ptr(k), v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  static DK void ev_wait(int k, int v) {
#ifdef DUCK_LAT_FORCE_TIMEOUT
    // test build (tests/test_gpu_env.py::test_latency_timeout_surfaces): workgroup 1's M event never
    // arrives for wave 3, whose wait for it gives up after a few polls
    const bool forced = blockIdx.x == 1 && k == EV_M;
    const int LIMIT = forced ? 1 << 6 : 1 << 20;
    if (forced) v += 1 << 24;
#else
    constexpr int LIMIT = 1 << 20;
#endif
    for (int it = 0; __hip_atomic_load(ev_ptr(k), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < v; it++) {
      if (it > LIMIT) {
        if ((threadIdx.x & 63) == 0) atomicAdd(&g_lat_timeouts, 1u);
        __hip_atomic_store(ev_ptr(EV_TIMEOUT), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  // did a wait of env set g give up (after the final barrier: every wave's waits are over)
  static DK bool ev_timed_out(int g) {
    extern __shared__ float lds_dyn[];
    return ((lds_int*)(lds_dyn + TL::EV))[4 * (EV_TIMEOUT + TL::NEV_G * g)] != 0;
  }
  // wave 0, substep s: kinematics and com_pos (everything else waits for them), rne's velocities
  // (the contact rows need the feet's), then the rest of rne and the actuation (qfrc_smooth)
  static DK void lat_r0(LP L, int lane, int s) {
    ev_wait(EV_EULER, s);
    LAT_T(0, s);
    kinematics(L, lane);
    com_pos(L, lane);
    ev_signal(EV_KIN, s + 1);
    LAT_T(1, s);
    rne_vel(L, lane);
    ev_signal(EV_VEL, s + 1);
    LAT_T(2, s);
    rne_rest<1>(L, lane);
    smooth(L, lane);
    ev_signal(EV_FSM, s + 1);
    LAT_T(3, s);
  }
  // wave 1: composite inertias and M (crb) while wave 0 finishes rne; M's register columns and the warm
  // start's products of qacc_warmstart while wave 3 factors M and solves for qacc_smooth; then the rest
  // of the warm start, the Newton solve, sensors, Euler
  static DK void lat_r1(LP L, int lane, int s, bool integrate, bool want_out, float* scratch, int sstride) {
    ev_wait(EV_KIN, s + 1);
    LAT_T(10, s);
    subtree_sums<2>(L, lane);
    crb(L, lane);
    ev_signal(EV_M, s + 1);
    LAT_T(11, s);
    {
      float Mc[NC][NV];
      load_cols(L, lane, Mc, false);
      LAT_T(12, s);
      float SL[6], SR[6], cwp;
      warm_start_a0(L, lane, Mc, SL, SR);
      ev_wait(EV_ROWS, s + 1);
      LAT_T(13, s);
      warm_start_a1(L, lane, SL, SR, cwp);
      ev_signal(EV_WA, s + 1);
      LAT_T(14, s);
      ev_wait(EV_QSM, s + 1);
      LAT_T(15, s);
      bool warm;
      const float g0 = warm_start_b(L, lane, cwp, warm);
      LAT_T(16, s);
      // every team starts from qacc_warmstart (the common case): wave 3 has computed the Newton direction
      // there meanwhile; otherwise this wave computes it (no wait)
      bool pre = false;
      if (__ballot(!warm) == 0ull) {
        ev_wait(EV_DIR, s + 1);
        pre = L[TL::XDIR + NV] != 0.0f;
      }
      LAT_T(19, s);
      newton(L, lane, scratch, sstride, Mc, g0, pre);
      LAT_T(17, s);
    }
    if (want_out) sensors(L, lane);
    if (integrate) {
      euler(L, lane);
    } else {
      team_for<NV>(lane, [&](int i) { L[Ly::WARM + i] = L[Ly::QACC + i]; });
      TSYNC();
    }
    ev_signal(EV_EULER, s + 1);
    LAT_T(18, s);
  }
  // wave 2: collision (kinematics only), then the constraint rows (the feet's velocities)
  static DK void lat_r2(LP L, int lane, int s, const float* hf) {
    ev_wait(EV_KIN, s + 1);
    LAT_T(20, s);
    collision(L, lane, hf);
    LAT_T(21, s);
    ev_wait(EV_VEL, s + 1);
    LAT_T(22, s);
    make_rows(L, lane);
    ev_signal(EV_ROWS, s + 1);
    LAT_T(23, s);
  }
  // wave 3: qacc_smooth = M^-1 qfrc_smooth from its own register columns of M
  static DK void lat_r3(LP L, int lane, int s) {
    ev_wait(EV_M, s + 1);
    LAT_T(30, s);
    float Mc[NC][NV];
    load_cols(L, lane, Mc, false);
    Fac F;
    smooth_factor(F, lane, Mc);
    LAT_T(31, s);
    ev_wait(EV_FSM, s + 1);
    LAT_T(32, s);
    smooth_solve(L, lane, F);
    ev_signal(EV_QSM, s + 1);
    LAT_T(33, s);
    // the Newton direction at qacc_warmstart, speculatively (wave 1 uses it when the warm start wins
    // everywhere in the wave): the rows' values there and M qacc_warmstart come from wave 1's warm start
    ev_wait(EV_WA, s + 1);
    LAT_T(34, s);
    const bool ok = newton_fused<false, TL::XDIR>(L, lane, Mc);
    if (lane == 0) L[TL::XDIR + NV] = ok ? 1.0f : 0.0f;
    TSYNC();
    ev_signal(EV_DIR, s + 1);
    LAT_T(35, s);
  }

  // ---------------- paired latency mode: one substep over two waves (step_kernel_lat<Md, 2>) ----------------
  // The same stages, events and scratch regions as the four-wave split (lat_r0 .. lat_r3), folded
  // onto two waves so that 8 envs per workgroup fill the chip at 2,048 envs (one wave per SIMD):
  // wave A (the env code's wave) takes kinematics, com_pos, rne and the actuation, then collision and
  // the constraint rows, then the speculative Newton direction at qacc_warmstart; wave B takes the
  // composite inertias, crb, M's register columns, the warm start's qacc_warmstart products, M's
  // factorization, the smooth solve, the rest of the warm start, the Newton step and line search,
  // sensors and Euler. Each wave's stages run in the order of their inputs, so B's chain is the
  // critical path: kinematics (A) -> crb -> ... -> the rows (A) -> warm start -> line search -> Euler.
  static DK void lat2_a(LP L, int lane, int s, const float* hf) {
    ev_wait(EV_EULER, s);
    LAT2_T(0, s);
    kinematics(L, lane);
    com_pos(L, lane);
    ev_signal(EV_KIN, s + 1);
    LAT2_T(1, s);
    rne_vel(L, lane);
    LAT2_T(2, s);
    rne_rest<1>(L, lane);
    smooth(L, lane);
    ev_signal(EV_FSM, s + 1);
    LAT2_T(3, s);
    collision(L, lane, hf);
    LAT2_T(4, s);
    make_rows(L, lane);
    ev_signal(EV_ROWS, s + 1);
    LAT2_T(5, s);
    // the Newton direction at qacc_warmstart, speculatively (B takes it when every team of the wave
    // starts there): M's columns from B's crb, the rows' values there and M qacc_warmstart from B's
    // warm start
    ev_wait(EV_M, s + 1);
    LAT2_T(6, s);
    float Mc[NC][NV];
    load_cols(L, lane, Mc, false);
    ev_wait(EV_WA, s + 1);
    LAT2_T(7, s);
    const bool ok = newton_fused<false, TL::XDIR>(L, lane, Mc);
    if (lane == 0) L[TL::XDIR + NV] = ok ? 1.0f : 0.0f;
    TSYNC();
    ev_signal(EV_DIR, s + 1);
    LAT2_T(8, s);
  }
  static DK void lat2_b(LP L, int lane, int s, bool integrate, bool want_out, float* scratch, int sstride) {
    ev_wait(EV_KIN, s + 1);
    LAT2_T(10, s);
    subtree_sums<2>(L, lane);
    crb(L, lane);
    ev_signal(EV_M, s + 1);
    LAT2_T(11, s);
    {
      float Mc[NC][NV];
      load_cols(L, lane, Mc, false);
      LAT2_T(12, s);
      float SL[6], SR[6], cwp;
      warm_start_a0(L, lane, Mc, SL, SR);
      LAT2_T(13, s);
      {
        Fac F;
        smooth_factor(F, lane, Mc);
        LAT2_T(14, s);
        ev_wait(EV_FSM, s + 1);
        LAT2_T(15, s);
        smooth_solve(L, lane, F);
        LAT2_T(16, s);
      }
      ev_wait(EV_ROWS, s + 1);
      LAT2_T(17, s);
      warm_start_a1(L, lane, SL, SR, cwp);
      ev_signal(EV_WA, s + 1);
      LAT2_T(18, s);
      bool warm;
      const float g0 = warm_start_b(L, lane, cwp, warm);
      LAT2_T(19, s);
      bool pre = false;
      if (__ballot(!warm) == 0ull) {
        ev_wait(EV_DIR, s + 1);
        pre = L[TL::XDIR + NV] != 0.0f;
      }
      LAT2_T(20, s);
      newton(L, lane, scratch, sstride, Mc, g0, pre);
      LAT2_T(21, s);
    }
    if (want_out) sensors(L, lane);
    if (integrate) {
      euler(L, lane);
    } else {
      team_for<NV>(lane, [&](int i) { L[Ly::WARM + i] = L[Ly::QACC + i]; });
      TSYNC();
    }
    LAT2_T(22, s);
    ev_signal(EV_EULER, s + 1);
  }
};
