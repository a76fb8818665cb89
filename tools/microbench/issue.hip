// Microbenchmark: VALU issue rate of ONE wave per SIMD vs two, per
// instruction class, independent and dependent streams (the regime of the
// quad/oct verify kernels at 10k signatures and below: one issue-bound wave
// per SIMD).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/microbench/issue tools/microbench/issue.hip
//
// Each variant is one inline-asm block: s_memtime, a loop of ITERS x 16
// instructions of one pattern, s_memtime. A workgroup of 64 x W threads puts
// W / 4 waves on every SIMD of one CU (W = 4: one wave per SIMD, W = 8: two).
// Prints cycles per instruction per wave (s_memtime counts at the shader
// clock's reference rate; only ratios between rows matter).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define R16(x) x x x x x x x x x x x x x x x x

#define BODY_ADD_IND                                                                                    \
  "v_add_u32 v100, v100, v140\n v_add_u32 v101, v101, v140\n v_add_u32 v102, v102, v140\n"              \
  "v_add_u32 v103, v103, v140\n v_add_u32 v104, v104, v140\n v_add_u32 v105, v105, v140\n"              \
  "v_add_u32 v106, v106, v140\n v_add_u32 v107, v107, v140\n v_add_u32 v108, v108, v140\n"              \
  "v_add_u32 v109, v109, v140\n v_add_u32 v110, v110, v140\n v_add_u32 v111, v111, v140\n"              \
  "v_add_u32 v112, v112, v140\n v_add_u32 v113, v113, v140\n v_add_u32 v114, v114, v140\n"              \
  "v_add_u32 v115, v115, v140\n"
#define BODY_ADD_DEP R16("v_add_u32 v100, v100, v140\n")
#define MAD(d) "v_mad_u64_u32 v[" #d ":" #d "+1], vcc, v140, v141, v[" #d ":" #d "+1]\n"
#define BODY_MAD_IND                                                                                    \
  "v_mad_u64_u32 v[100:101], vcc, v140, v141, v[100:101]\n v_mad_u64_u32 v[102:103], vcc, v140, v141, v[102:103]\n" \
  "v_mad_u64_u32 v[104:105], vcc, v140, v141, v[104:105]\n v_mad_u64_u32 v[106:107], vcc, v140, v141, v[106:107]\n" \
  "v_mad_u64_u32 v[108:109], vcc, v140, v141, v[108:109]\n v_mad_u64_u32 v[110:111], vcc, v140, v141, v[110:111]\n" \
  "v_mad_u64_u32 v[112:113], vcc, v140, v141, v[112:113]\n v_mad_u64_u32 v[114:115], vcc, v140, v141, v[114:115]\n" \
  "v_mad_u64_u32 v[100:101], vcc, v140, v141, v[100:101]\n v_mad_u64_u32 v[102:103], vcc, v140, v141, v[102:103]\n" \
  "v_mad_u64_u32 v[104:105], vcc, v140, v141, v[104:105]\n v_mad_u64_u32 v[106:107], vcc, v140, v141, v[106:107]\n" \
  "v_mad_u64_u32 v[108:109], vcc, v140, v141, v[108:109]\n v_mad_u64_u32 v[110:111], vcc, v140, v141, v[110:111]\n" \
  "v_mad_u64_u32 v[112:113], vcc, v140, v141, v[112:113]\n v_mad_u64_u32 v[114:115], vcc, v140, v141, v[114:115]\n"
#define BODY_MAD_DEP R16("v_mad_u64_u32 v[100:101], vcc, v140, v141, v[100:101]\n")
// mad whose 32-bit multiplicand is the previous mad's low word (a real
// dependency through the multiplier input, as in a carry chain)
#define BODY_MAD_DEP_MUL R16("v_mad_u64_u32 v[100:101], vcc, v100, v141, v[102:103]\n")
#define BODY_SHR64_IND                                                                                  \
  "v_lshrrev_b64 v[100:101], 26, v[116:117]\n v_lshrrev_b64 v[102:103], 26, v[118:119]\n"               \
  "v_lshrrev_b64 v[104:105], 26, v[120:121]\n v_lshrrev_b64 v[106:107], 26, v[122:123]\n"               \
  "v_lshrrev_b64 v[108:109], 26, v[124:125]\n v_lshrrev_b64 v[110:111], 26, v[126:127]\n"               \
  "v_lshrrev_b64 v[112:113], 26, v[128:129]\n v_lshrrev_b64 v[114:115], 26, v[130:131]\n"               \
  "v_lshrrev_b64 v[100:101], 26, v[116:117]\n v_lshrrev_b64 v[102:103], 26, v[118:119]\n"               \
  "v_lshrrev_b64 v[104:105], 26, v[120:121]\n v_lshrrev_b64 v[106:107], 26, v[122:123]\n"               \
  "v_lshrrev_b64 v[108:109], 26, v[124:125]\n v_lshrrev_b64 v[110:111], 26, v[126:127]\n"               \
  "v_lshrrev_b64 v[112:113], 26, v[128:129]\n v_lshrrev_b64 v[114:115], 26, v[130:131]\n"
// a carry link: c = h >> 26 (64-bit); h' += c -- dependent pairs
#define BODY_CARRY_DEP                                                                                  \
  R16("v_lshrrev_b64 v[102:103], 26, v[100:101]\n v_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\n")
#define BODY_ADD64_IND                                                                                  \
  "v_lshl_add_u64 v[100:101], v[116:117], 0, v[100:101]\n v_lshl_add_u64 v[102:103], v[116:117], 0, v[102:103]\n" \
  "v_lshl_add_u64 v[104:105], v[116:117], 0, v[104:105]\n v_lshl_add_u64 v[106:107], v[116:117], 0, v[106:107]\n" \
  "v_lshl_add_u64 v[108:109], v[116:117], 0, v[108:109]\n v_lshl_add_u64 v[110:111], v[116:117], 0, v[110:111]\n" \
  "v_lshl_add_u64 v[112:113], v[116:117], 0, v[112:113]\n v_lshl_add_u64 v[114:115], v[116:117], 0, v[114:115]\n" \
  "v_lshl_add_u64 v[100:101], v[116:117], 0, v[100:101]\n v_lshl_add_u64 v[102:103], v[116:117], 0, v[102:103]\n" \
  "v_lshl_add_u64 v[104:105], v[116:117], 0, v[104:105]\n v_lshl_add_u64 v[106:107], v[116:117], 0, v[106:107]\n" \
  "v_lshl_add_u64 v[108:109], v[116:117], 0, v[108:109]\n v_lshl_add_u64 v[110:111], v[116:117], 0, v[110:111]\n" \
  "v_lshl_add_u64 v[112:113], v[116:117], 0, v[112:113]\n v_lshl_add_u64 v[114:115], v[116:117], 0, v[114:115]\n"
#define BODY_MIX_IND                                                                                    \
  "v_mad_u64_u32 v[100:101], vcc, v140, v141, v[100:101]\n v_add_u32 v120, v120, v140\n"                \
  "v_mad_u64_u32 v[102:103], vcc, v140, v141, v[102:103]\n v_add_u32 v121, v121, v140\n"                \
  "v_mad_u64_u32 v[104:105], vcc, v140, v141, v[104:105]\n v_add_u32 v122, v122, v140\n"                \
  "v_mad_u64_u32 v[106:107], vcc, v140, v141, v[106:107]\n v_add_u32 v123, v123, v140\n"                \
  "v_mad_u64_u32 v[108:109], vcc, v140, v141, v[108:109]\n v_add_u32 v124, v124, v140\n"                \
  "v_mad_u64_u32 v[110:111], vcc, v140, v141, v[110:111]\n v_add_u32 v125, v125, v140\n"                \
  "v_mad_u64_u32 v[112:113], vcc, v140, v141, v[112:113]\n v_add_u32 v126, v126, v140\n"                \
  "v_mad_u64_u32 v[114:115], vcc, v140, v141, v[114:115]\n v_add_u32 v127, v127, v140\n"
#define BODY_DPP_IND                                                                                    \
  "v_mov_b32_dpp v100, v120 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                          \
  "v_mov_b32_dpp v101, v121 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                          \
  "v_mov_b32_dpp v102, v122 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                          \
  "v_mov_b32_dpp v103, v123 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                          \
  "v_mov_b32_dpp v104, v124 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                          \
  "v_mov_b32_dpp v105, v125 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                          \
  "v_mov_b32_dpp v106, v126 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                          \
  "v_mov_b32_dpp v107, v127 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                          \
  "v_mov_b32_dpp v108, v120 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                          \
  "v_mov_b32_dpp v109, v121 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                          \
  "v_mov_b32_dpp v110, v122 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                          \
  "v_mov_b32_dpp v111, v123 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                          \
  "v_mov_b32_dpp v112, v124 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                          \
  "v_mov_b32_dpp v113, v125 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                          \
  "v_mov_b32_dpp v114, v126 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                          \
  "v_mov_b32_dpp v115, v127 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define BODY_MULLO_IND                                                                                  \
  "v_mul_lo_u32 v100, v120, v140\n v_mul_lo_u32 v101, v121, v140\n v_mul_lo_u32 v102, v122, v140\n"     \
  "v_mul_lo_u32 v103, v123, v140\n v_mul_lo_u32 v104, v124, v140\n v_mul_lo_u32 v105, v125, v140\n"     \
  "v_mul_lo_u32 v106, v126, v140\n v_mul_lo_u32 v107, v127, v140\n v_mul_lo_u32 v108, v120, v140\n"     \
  "v_mul_lo_u32 v109, v121, v140\n v_mul_lo_u32 v110, v122, v140\n v_mul_lo_u32 v111, v123, v140\n"     \
  "v_mul_lo_u32 v112, v124, v140\n v_mul_lo_u32 v113, v125, v140\n v_mul_lo_u32 v114, v126, v140\n"     \
  "v_mul_lo_u32 v115, v127, v140\n"
// 32-bit mul pair (lo + hi) as a 32x32->64 product: independent
#define BODY_MULHI_IND                                                                                  \
  "v_mul_hi_u32 v100, v120, v140\n v_mul_hi_u32 v101, v121, v140\n v_mul_hi_u32 v102, v122, v140\n"     \
  "v_mul_hi_u32 v103, v123, v140\n v_mul_hi_u32 v104, v124, v140\n v_mul_hi_u32 v105, v125, v140\n"     \
  "v_mul_hi_u32 v106, v126, v140\n v_mul_hi_u32 v107, v127, v140\n v_mul_hi_u32 v108, v120, v140\n"     \
  "v_mul_hi_u32 v109, v121, v140\n v_mul_hi_u32 v110, v122, v140\n v_mul_hi_u32 v111, v123, v140\n"     \
  "v_mul_hi_u32 v112, v124, v140\n v_mul_hi_u32 v113, v125, v140\n v_mul_hi_u32 v114, v126, v140\n"     \
  "v_mul_hi_u32 v115, v127, v140\n"
// 24-bit mads (v_mad_u32_u24: 24x24 -> low 32 + add) independent
#define BODY_MAD24_IND                                                                                  \
  "v_mad_u32_u24 v100, v120, v140, v100\n v_mad_u32_u24 v101, v121, v140, v101\n"                       \
  "v_mad_u32_u24 v102, v122, v140, v102\n v_mad_u32_u24 v103, v123, v140, v103\n"                       \
  "v_mad_u32_u24 v104, v124, v140, v104\n v_mad_u32_u24 v105, v125, v140, v105\n"                       \
  "v_mad_u32_u24 v106, v126, v140, v106\n v_mad_u32_u24 v107, v127, v140, v107\n"                       \
  "v_mad_u32_u24 v108, v120, v140, v108\n v_mad_u32_u24 v109, v121, v140, v109\n"                       \
  "v_mad_u32_u24 v110, v122, v140, v110\n v_mad_u32_u24 v111, v123, v140, v111\n"                       \
  "v_mad_u32_u24 v112, v124, v140, v112\n v_mad_u32_u24 v113, v125, v140, v113\n"                       \
  "v_mad_u32_u24 v114, v126, v140, v114\n v_mad_u32_u24 v115, v127, v140, v115\n"
// packed 32-bit FMA (two lanes of f32 per instruction) independent
#define BODY_PKFMA_IND                                                                                  \
  "v_pk_fma_f32 v[100:101], v[120:121], v[140:141], v[100:101]\n"                                      \
  "v_pk_fma_f32 v[102:103], v[120:121], v[140:141], v[102:103]\n"                                      \
  "v_pk_fma_f32 v[104:105], v[120:121], v[140:141], v[104:105]\n"                                      \
  "v_pk_fma_f32 v[106:107], v[120:121], v[140:141], v[106:107]\n"                                      \
  "v_pk_fma_f32 v[108:109], v[120:121], v[140:141], v[108:109]\n"                                      \
  "v_pk_fma_f32 v[110:111], v[120:121], v[140:141], v[110:111]\n"                                      \
  "v_pk_fma_f32 v[112:113], v[120:121], v[140:141], v[112:113]\n"                                      \
  "v_pk_fma_f32 v[114:115], v[120:121], v[140:141], v[114:115]\n"                                      \
  "v_pk_fma_f32 v[100:101], v[122:123], v[140:141], v[100:101]\n"                                      \
  "v_pk_fma_f32 v[102:103], v[122:123], v[140:141], v[102:103]\n"                                      \
  "v_pk_fma_f32 v[104:105], v[122:123], v[140:141], v[104:105]\n"                                      \
  "v_pk_fma_f32 v[106:107], v[122:123], v[140:141], v[106:107]\n"                                      \
  "v_pk_fma_f32 v[108:109], v[122:123], v[140:141], v[108:109]\n"                                      \
  "v_pk_fma_f32 v[110:111], v[122:123], v[140:141], v[110:111]\n"                                      \
  "v_pk_fma_f32 v[112:113], v[122:123], v[140:141], v[112:113]\n"                                      \
  "v_pk_fma_f32 v[114:115], v[122:123], v[140:141], v[114:115]\n"

#define CLOBBERS                                                                                        \
  "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111",       \
      "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123",   \
      "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v140", "v141", "vcc", "s80",    \
      "s81", "s82", "s83", "s84", "scc"

#define KERNEL(name, BODY)                                                                              \
  __global__ __launch_bounds__(512) void name(uint32_t iters, uint64_t* out) {                          \
    uint32_t lo0, hi0, lo1, hi1, hw;                                                                    \
    asm volatile(                                                                                       \
        "v_mov_b32 v140, 3\n v_mov_b32 v141, 5\n"                                                       \
        "v_mov_b32 v116, 7\n v_mov_b32 v117, 0\n v_mov_b32 v118, 7\n v_mov_b32 v119, 0\n"              \
        "v_mov_b32 v120, 9\n v_mov_b32 v121, 9\n v_mov_b32 v122, 9\n v_mov_b32 v123, 9\n"              \
        "v_mov_b32 v124, 9\n v_mov_b32 v125, 9\n v_mov_b32 v126, 9\n v_mov_b32 v127, 9\n"              \
        "v_mov_b32 v128, 9\n v_mov_b32 v129, 0\n v_mov_b32 v130, 9\n v_mov_b32 v131, 0\n"              \
        "v_mov_b32 v100, 0\n v_mov_b32 v101, 0\n v_mov_b32 v102, 0\n v_mov_b32 v103, 0\n"              \
        "v_mov_b32 v104, 0\n v_mov_b32 v105, 0\n v_mov_b32 v106, 0\n v_mov_b32 v107, 0\n"              \
        "v_mov_b32 v108, 0\n v_mov_b32 v109, 0\n v_mov_b32 v110, 0\n v_mov_b32 v111, 0\n"              \
        "v_mov_b32 v112, 0\n v_mov_b32 v113, 0\n v_mov_b32 v114, 0\n v_mov_b32 v115, 0\n"              \
        "s_mov_b32 s84, %5\n"                                                                          \
        "s_memtime s[80:81]\n s_waitcnt lgkmcnt(0)\n"                                                 \
        "1:\n" BODY                                                                                     \
        "s_sub_u32 s84, s84, 1\n s_cmp_lg_u32 s84, 0\n s_cbranch_scc1 1b\n"                         \
        "s_memtime s[82:83]\n s_waitcnt lgkmcnt(0)\n"                                                 \
        "s_getreg_b32 s85, hwreg(HW_REG_HW_ID)\n"                                                      \
        "v_mov_b32 %0, s80\n v_mov_b32 %1, s81\n v_mov_b32 %2, s82\n v_mov_b32 %3, s83\n"          \
        "v_mov_b32 %4, s85\n"                                                                          \
        : "=v"(lo0), "=v"(hi0), "=v"(lo1), "=v"(hi1), "=v"(hw)                                          \
        : "s"(iters)                                                                                    \
        : CLOBBERS, "s85");                                                                             \
    if ((threadIdx.x & 63) == 0) {                                                                      \
      const uint64_t t0 = ((uint64_t)hi0 << 32) | lo0, t1 = ((uint64_t)hi1 << 32) | lo1;                \
      out[2 * (threadIdx.x >> 6)] = t1 - t0;                                                            \
      out[2 * (threadIdx.x >> 6) + 1] = hw;                                                             \
    }                                                                                                   \
  }

KERNEL(k_add_ind, BODY_ADD_IND)
KERNEL(k_add_dep, BODY_ADD_DEP)
KERNEL(k_mad_ind, BODY_MAD_IND)
KERNEL(k_mad_dep, BODY_MAD_DEP)
KERNEL(k_mad_dep_mul, BODY_MAD_DEP_MUL)
KERNEL(k_shr64_ind, BODY_SHR64_IND)
KERNEL(k_carry_dep, BODY_CARRY_DEP)
KERNEL(k_add64_ind, BODY_ADD64_IND)
KERNEL(k_mix_ind, BODY_MIX_IND)
KERNEL(k_dpp_ind, BODY_DPP_IND)
KERNEL(k_mullo_ind, BODY_MULLO_IND)
KERNEL(k_mulhi_ind, BODY_MULHI_IND)
KERNEL(k_mad24_ind, BODY_MAD24_IND)
KERNEL(k_pkfma_ind, BODY_PKFMA_IND)

typedef void (*Kern)(uint32_t, uint64_t*);

int main() {
  struct V {
    const char* name;
    Kern k;
    int insts;  // instructions per loop body
  } vs[] = {{"v_add_u32 indep", k_add_ind, 16},
            {"v_add_u32 dep", k_add_dep, 16},
            {"v_mad_u64_u32 indep (8 acc)", k_mad_ind, 16},
            {"v_mad_u64_u32 dep (accumulator)", k_mad_dep, 16},
            {"v_mad_u64_u32 dep (multiplicand)", k_mad_dep_mul, 16},
            {"v_lshrrev_b64 indep", k_shr64_ind, 16},
            {"carry link shr64+lshl_add dep", k_carry_dep, 32},
            {"v_lshl_add_u64 indep", k_add64_ind, 16},
            {"mad64 + add32 interleaved indep", k_mix_ind, 16},
            {"v_mov_b32_dpp indep", k_dpp_ind, 16},
            {"v_mul_lo_u32 indep", k_mullo_ind, 16},
            {"v_mul_hi_u32 indep", k_mulhi_ind, 16},
            {"v_mad_u32_u24 indep", k_mad24_ind, 16},
            {"v_pk_fma_f32 indep", k_pkfma_ind, 16}};
  const uint32_t iters = 4096;
  uint64_t* d = nullptr;
  if (hipMalloc(&d, 8 * 32) != hipSuccess) return 1;
  std::printf("# cycles (s_memtime) per instruction per wave, by workgroup size (waves); [simd ids]\n");
  for (const V& v : vs) {
    std::printf("%-36s", v.name);
    for (int waves : {1, 2, 4, 8}) {
      hipLaunchKernelGGL(v.k, dim3(1), dim3(64 * waves), 0, 0, iters, d);  // warm-up
      hipLaunchKernelGGL(v.k, dim3(1), dim3(64 * waves), 0, 0, iters, d);
      std::vector<uint64_t> h(2 * waves);
      if (hipMemcpy(h.data(), d, 16 * waves, hipMemcpyDeviceToHost) != hipSuccess) return 1;
      double mx = 0;
      char ids[64];
      int o = 0;
      for (int w = 0; w < waves; w++) {
        mx = (double)h[2 * w] > mx ? (double)h[2 * w] : mx;
        o += std::snprintf(ids + o, sizeof(ids) - o, "%d", (int)((h[2 * w + 1] >> 4) & 3));  // HW_ID simd_id
      }
      std::printf("  %dw %6.2f [%s]", waves, mx / ((double)iters * v.insts), ids);
    }
    std::printf("\n");
  }
  (void)hipFree(d);
  return 0;
}
