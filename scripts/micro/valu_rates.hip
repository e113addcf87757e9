// Issue cost of single VALU instructions on gfx950, one wave per SIMD and four waves per SIMD: each lane runs
// 8 independent chains of N instructions of one kind (inline asm, so the compiler neither folds nor vectorizes),
// timed with s_memtime inside the kernel.  Used to price the instructions of the f16-derivative experiment
// (VISSM_DERIV16: v_fma_mix_f32, v_cvt_pk_f16_f32, v_exp_f32 with clamp) against the forms they replaced.
// build: hipcc -O3 --offload-arch=gfx950 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 256
#define BODY(INSTR)                                                                                      \
  _Pragma("unroll 1") for (int i = 0; i < N; ++i) {                                                      \
    asm volatile(INSTR : "+v"(a0) : "v"(b) : );                                                          \
    asm volatile(INSTR : "+v"(a1) : "v"(b) : );                                                          \
    asm volatile(INSTR : "+v"(a2) : "v"(b) : );                                                          \
    asm volatile(INSTR : "+v"(a3) : "v"(b) : );                                                          \
    asm volatile(INSTR : "+v"(a4) : "v"(b) : );                                                          \
    asm volatile(INSTR : "+v"(a5) : "v"(b) : );                                                          \
    asm volatile(INSTR : "+v"(a6) : "v"(b) : );                                                          \
    asm volatile(INSTR : "+v"(a7) : "v"(b) : );                                                          \
  }
template <int K>
__global__ void kern(float* out, long long* cyc, float seed) {
  float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
        a7 = a0 + 7, b = 0.5f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  if constexpr (K == 0) BODY("v_fma_f32 %0, %0, %1, %1")
  if constexpr (K == 1) BODY("v_fma_mix_f32 %0, %0, %1, 0 op_sel_hi:[0,1,0]")
  if constexpr (K == 2) BODY("v_cvt_pk_f16_f32 %0, %0, %1")
  if constexpr (K == 3) BODY("v_exp_f32 %0, %0")
  if constexpr (K == 4) BODY("v_exp_f32_e64 %0, %0 clamp")
  if constexpr (K == 5) BODY("v_cvt_pk_bf16_f32 %0, %0, %1")
  if constexpr (K == 6) BODY("v_med3_f32 %0, %0, %1, 1.0")
  if constexpr (K == 7) BODY("v_cvt_f32_f16 %0, %0")
  if constexpr (K == 8) BODY("v_mul_f32 %0, %0, %1")
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int K>
void run(const char* name, int wps) {
  float* out; long long* cyc;
  const int blocks = 256 * 4 * wps;  // 64-thread blocks: wps waves per SIMD
  hipMalloc(&out, blocks * 64 * 4); hipMalloc(&cyc, blocks * 8);
  hipLaunchKernelGGL(kern<K>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1.f);
  hipDeviceSynchronize();
  long long* h = new long long[blocks];
  hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
  double s = 0; for (int i = 0; i < blocks; ++i) s += h[i];
  printf("%-26s waves/SIMD %d: %.2f memtime ticks per instruction per wave\n", name, wps, s / blocks / (8.0 * N));
  hipFree(out); hipFree(cyc); delete[] h;
}
int main() {
  for (int wps : {1, 4}) {
    run<0>("v_fma_f32", wps); run<1>("v_fma_mix_f32", wps); run<2>("v_cvt_pk_f16_f32", wps);
    run<3>("v_exp_f32", wps); run<4>("v_exp_f32 clamp", wps); run<5>("v_cvt_pk_bf16_f32", wps);
    run<6>("v_med3_f32", wps); run<7>("v_cvt_f32_f16", wps); run<8>("v_mul_f32", wps);
  }
  return 0;
}
