// issue_probe.hip -- issue cost of VALU instruction kinds for ONE wave alone on its SIMD, and for
// several waves of one block, the regime of the RK45 straggler tail.  Each probe runs
// a loop of 16 instructions of one kind (8 independent chains, or 1 dependent chain) and reports
// shader cycles per instruction per wave from s_memtime.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/issue_probe tools/issue_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define ITERS 4096
#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define R16(X) R8(X) R8(X)

typedef float f2 __attribute__((ext_vector_type(2)));

template <int K>
__global__ void probe(float* out, long long* cyc, float seed) {
  float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
        a7 = a0 + 7;
  const float b = seed * 0.5f, c = seed * 0.25f;
  f2 p0 = {a0, a1}, p1 = {a1, a2}, p2 = {a2, a3}, p3 = {a3, a4}, p4 = {a4, a5}, p5 = {a5, a6}, p6 = {a6, a7},
     p7 = {a7, a0};
  const f2 pb = {b, c}, pc = {c, b};
  double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7;
  const double db = b, dc = c;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; i++) {
#define FMA_I(j) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a##j) : "v"(b), "v"(c));
#define FMA_D(j) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));
#define DPP_I(j) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a##j));
#define EXP_I(j) asm volatile("v_exp_f32 %0, %0" : "+v"(a##j));
#define EXP_D(j) asm volatile("v_exp_f32 %0, %0" : "+v"(a0));
#define CND_I(j) asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(a##j) : "v"(b), "s"(0x5555555555555555ull));
#define PK_I(j) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p##j) : "v"(pb), "v"(pc));
#define PK_D(j) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p0) : "v"(pb), "v"(pc));
#define F64_I(j) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d##j) : "v"(db), "v"(dc));
#define ADPP_I(j) asm volatile("v_add_f32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a##j) : "v"(b));
#define DPPFMA_D(j) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 1\n\tv_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));
#define MIX_I(j) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a##j) : "v"(b), "v"(c)); \
                 asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p##j) : "v"(pb), "v"(pc));
    if constexpr (K == 0) { R16(FMA_I) }
    else if constexpr (K == 1) { R16(FMA_D) }
    else if constexpr (K == 2) { R16(DPP_I) }
    else if constexpr (K == 3) { R16(EXP_I) }
    else if constexpr (K == 4) { R16(EXP_D) }
    else if constexpr (K == 5) { R16(CND_I) }
    else if constexpr (K == 6) { R16(PK_I) }
    else if constexpr (K == 7) { R16(PK_D) }
    else if constexpr (K == 8) { R16(F64_I) }
    else if constexpr (K == 9) { R16(ADPP_I) }
    else if constexpr (K == 10) { R8(DPPFMA_D) }  // 8 pairs (+ s_nop 1): 16 VALU
    else if constexpr (K == 11) { R8(MIX_I) }     // 8 fma + 8 pk_fma interleaved
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  s += p0.x + p1.y + p2.x + p3.y + p4.x + p5.y + p6.x + p7.y + p0.y + p7.x;
  s += (float)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

static const char* NAMES[] = {"v_fma_f32 indep",     "v_fma_f32 dep",      "v_mov_b32_dpp indep", "v_exp_f32 indep",
                              "v_exp_f32 dep",       "v_cndmask indep",    "v_pk_fma_f32 indep",  "v_pk_fma_f32 dep",
                              "v_fma_f64 indep",     "v_add_f32_dpp indep", "dpp->fma dep (+s_nop1)", "fma+pk_fma mix"};

template <int K>
void run(int threads) {
  float* out;
  long long* cyc;
  const int waves = threads / 64;
  hipMalloc(&out, threads * sizeof(float));
  hipMalloc(&cyc, waves * sizeof(long long));
  hipLaunchKernelGGL(probe<K>, dim3(1), dim3(threads), 0, 0, out, cyc, 1.0f);  // warm
  hipLaunchKernelGGL(probe<K>, dim3(1), dim3(threads), 0, 0, out, cyc, 1.0f);
  hipDeviceSynchronize();
  std::vector<long long> h(waves);
  hipMemcpy(h.data(), cyc, waves * sizeof(long long), hipMemcpyDeviceToHost);
  long long mx = 0;
  for (long long v : h) mx = v > mx ? v : mx;
  // s_memtime counts at the constant 100 MHz reference on some parts; report raw and per-instruction
  printf("%-24s waves/block %2d  ticks %9lld  ticks/instr %.3f\n", NAMES[K], waves, mx, (double)mx / (ITERS * 16.0));
  hipFree(out);
  hipFree(cyc);
}

template <int K>
void all() {
  run<K>(64);
  run<K>(256);
  run<K>(512);
}

int main() {
  all<0>(); all<1>(); all<2>(); all<3>(); all<4>(); all<5>(); all<6>(); all<7>(); all<8>(); all<9>(); all<10>(); all<11>();
  return 0;
}
