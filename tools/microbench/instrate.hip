// Per-instruction VALU issue rate on gfx950 for the integer ops the CKKS kernels are built from.
// Each kernel runs 8 independent chains of one instruction per thread; rate = wave-instructions
// per CU-cycle derived from the measured time and the reported shader clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1;}}while(0)

#define BODY8(INS) INS(a0) INS(a1) INS(a2) INS(a3) INS(a4) INS(a5) INS(a6) INS(a7)

__global__ void k_mad64(uint64_t* out, uint32_t b, int iters) {
  uint64_t a0=threadIdx.x,a1=a0+1,a2=a0+2,a3=a0+3,a4=a0+4,a5=a0+5,a6=a0+6,a7=a0+7;
  for (int i=0;i<iters;++i) {
#define I(x) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(x) : "v"((uint32_t)x), "v"(b) : "s40", "s41");
    BODY8(I)
#undef I
  }
  out[blockIdx.x*blockDim.x+threadIdx.x]=a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ void k_mullo(uint64_t* out, uint32_t b, int iters) {
  uint32_t a0=threadIdx.x,a1=a0+1,a2=a0+2,a3=a0+3,a4=a0+4,a5=a0+5,a6=a0+6,a7=a0+7;
  for (int i=0;i<iters;++i) {
#define I(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
    BODY8(I)
#undef I
  }
  out[blockIdx.x*blockDim.x+threadIdx.x]=a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ void k_mulhi(uint64_t* out, uint32_t b, int iters) {
  uint32_t a0=threadIdx.x,a1=a0+1,a2=a0+2,a3=a0+3,a4=a0+4,a5=a0+5,a6=a0+6,a7=a0+7;
  for (int i=0;i<iters;++i) {
#define I(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(b));
    BODY8(I)
#undef I
  }
  out[blockIdx.x*blockDim.x+threadIdx.x]=a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ void k_mul24(uint64_t* out, uint32_t b, int iters) {
  uint32_t a0=threadIdx.x,a1=a0+1,a2=a0+2,a3=a0+3,a4=a0+4,a5=a0+5,a6=a0+6,a7=a0+7;
  for (int i=0;i<iters;++i) {
#define I(x) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(b));
    BODY8(I)
#undef I
  }
  out[blockIdx.x*blockDim.x+threadIdx.x]=a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ void k_add(uint64_t* out, uint32_t b, int iters) {
  uint32_t a0=threadIdx.x,a1=a0+1,a2=a0+2,a3=a0+3,a4=a0+4,a5=a0+5,a6=a0+6,a7=a0+7;
  for (int i=0;i<iters;++i) {
#define I(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
    BODY8(I)
#undef I
  }
  out[blockIdx.x*blockDim.x+threadIdx.x]=a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ void k_add64(uint64_t* out, uint32_t b, int iters) {
  uint64_t a0=threadIdx.x,a1=a0+1,a2=a0+2,a3=a0+3,a4=a0+4,a5=a0+5,a6=a0+6,a7=a0+7; uint64_t bb=b;
  for (int i=0;i<iters;++i) {
#define I(x) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(x) : "v"(bb));
    BODY8(I)
#undef I
  }
  out[blockIdx.x*blockDim.x+threadIdx.x]=a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ void k_fma64(uint64_t* out, uint32_t b, int iters) {
  double a0=threadIdx.x,a1=a0+1,a2=a0+2,a3=a0+3,a4=a0+4,a5=a0+5,a6=a0+6,a7=a0+7; double bb=1.0000001*b;
  for (int i=0;i<iters;++i) {
#define I(x) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(x) : "v"(bb));
    BODY8(I)
#undef I
  }
  out[blockIdx.x*blockDim.x+threadIdx.x]=(uint64_t)(a0+a1+a2+a3+a4+a5+a6+a7);
}

int main() {
  uint64_t* d; CK(hipMalloc(&d, 64<<20));
  int clk=0; hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  hipEvent_t a,b; hipEventCreate(&a); hipEventCreate(&b);
  const int blocks=256*8, threads=256, iters=4000;
  struct { const char* n; void (*k)(uint64_t*, uint32_t, int); } ks[] = {
    {"v_mad_u64_u32", k_mad64}, {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi},
    {"v_mul_u32_u24", k_mul24}, {"v_add_u32", k_add}, {"v_lshl_add_u64", k_add64}, {"v_fma_f64", k_fma64}};
  printf("clock %d kHz\n", clk);
  for (int rep=0; rep<2; ++rep) for (auto& k : ks) {
    float ms;
    hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), 0, 0, d, 12345u, 10);
    hipEventRecord(a); hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), 0, 0, d, 12345u, iters); hipEventRecord(b);
    hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    double winst = (double)blocks*threads/64*iters*8;             // wave-instructions
    double cyc = ms*1e-3 * clk*1e3 * 256 * 4;                       // SIMD-cycles available
    printf("%-16s %8.3f ms  %6.2f cycles/wave-instr/SIMD  %.2e lane-ops/s\n", k.n, ms, cyc/winst, winst*64/(ms*1e-3));
  }
  return 0;
}
