// valu_probe.hip -- issue cost of the RS kernels' VALU mix on MI355X: v_perm_b32,
// v_bitop3_b32, v_and_b32 / v_lshrrev_b32, each in 8 independent chains, at 1..8
// waves per SIMD (one 256-thread block per CU per 4 waves... see grid below).
// Prints wave-instructions per cycle per CU from hipEvent time and the clock.
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_probe valu_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;

template <int OP>
__global__ __launch_bounds__(256) void probe(uint32_t* out, uint32_t seed) {
  uint32_t v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = seed * (threadIdx.x + 1) + i * 0x01010101u;
  uint32_t t0 = __builtin_amdgcn_readfirstlane(seed ^ 0x12345678u), t1 = __builtin_amdgcn_readfirstlane(seed + 7);
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (OP == 0) v[i] = __builtin_amdgcn_perm(t1, v[i], v[(i + 1) & 7] & 0x07070707u);  // perm + and
      if constexpr (OP == 1) v[i] = __builtin_amdgcn_bitop3_b32(v[i], v[(i + 3) & 7], t0, 0x96);
      if constexpr (OP == 2) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[i]) : "v"(v[(i + 5) & 7]));
      if constexpr (OP == 3) v[i] = __builtin_amdgcn_perm(t1, t0, v[i]);  // perm only (sel = data)
      if constexpr (OP == 4) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(v[i]));
      if constexpr (OP == 5) asm volatile("v_and_b32 %0, %1, %0" : "+v"(v[i]) : "v"(v[(i + 5) & 7]));
      if constexpr (OP == 6) asm volatile("v_bfi_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(v[(i + 5) & 7]), "v"(v[(i + 3) & 7]));
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc ^= v[i];
  if (acc == 0xDEADBEEFu) out[threadIdx.x] = acc;
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  uint32_t* out;
  (void)hipMalloc(&out, 4096);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[] = {"v_perm+v_and (2 instr)", "v_bitop3", "v_xor_b32", "v_perm", "v_lshlrev_b32", "v_and_b32", "v_bfi_b32"};
  const int per_iter[] = {16, 8, 8, 8, 8, 8, 8};
  for (int op = 0; op < 7; ++op) {
    for (int wps : {1, 2, 4, 8}) {  // waves per SIMD: wps*4 waves per CU = wps blocks of 256
      const int grid = cus * wps;
      auto launch = [&] {
        if (op == 0) hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(256), 0, 0, out, 3u);
        if (op == 1) hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(256), 0, 0, out, 3u);
        if (op == 2) hipLaunchKernelGGL(probe<2>, dim3(grid), dim3(256), 0, 0, out, 3u);
        if (op == 3) hipLaunchKernelGGL(probe<3>, dim3(grid), dim3(256), 0, 0, out, 3u);
        if (op == 4) hipLaunchKernelGGL(probe<4>, dim3(grid), dim3(256), 0, 0, out, 3u);
        if (op == 5) hipLaunchKernelGGL(probe<5>, dim3(grid), dim3(256), 0, 0, out, 3u);
        if (op == 6) hipLaunchKernelGGL(probe<6>, dim3(grid), dim3(256), 0, 0, out, 3u);
      };
      launch();
      (void)hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double s = ms / 5 * 1e-3;
      const double winstr = static_cast<double>(grid) * 4 * kIters * per_iter[op];  // wave-instructions
      const double clk = 2.4e9;
      printf("%-28s waves/SIMD=%d: %.3f wave-instr/cycle/CU (peak 2 at 2 cyc/instr/SIMD)  %.1f us\n", names[op],
             wps, winstr / s / clk / cus, s * 1e6);
    }
  }
  return 0;
}
