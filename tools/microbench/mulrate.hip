// Microbenchmark: 64-bit modular multiply throughput on gfx950 (Shoup / full 128-bit product),
// plus a plain u64 streaming copy for an HBM reference. Used to size the NTT/Hadamard design.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1;}}while(0)
typedef unsigned long long u64;

__global__ void k_shoup(u64* out, u64 w, u64 wp, u64 q, int iters) {
  u64 y[8];
  for (int k=0;k<8;k++) y[k] = threadIdx.x*8+k + blockIdx.x;
  for (int it=0; it<iters; ++it) {
    #pragma unroll
    for (int k=0;k<8;k++) {
      u64 qh = __umul64hi(wp, y[k]);
      y[k] = w*y[k] - qh*q;
    }
  }
  u64 s=0; for(int k=0;k<8;k++) s^=y[k];
  out[blockIdx.x*blockDim.x+threadIdx.x]=s;
}
__global__ void k_mul128(u64* out, u64 b, int iters) {
  u64 lo[8], hi[8], a[8];
  for (int k=0;k<8;k++){ a[k] = threadIdx.x*8+k + blockIdx.x; lo[k]=0; hi[k]=0; }
  for (int it=0; it<iters; ++it) {
    #pragma unroll
    for (int k=0;k<8;k++) {
      u64 l = a[k]*b; u64 h = __umul64hi(a[k], b);
      lo[k] += l; hi[k] += h + (lo[k] < l);
      a[k] ^= h;
    }
  }
  u64 s=0; for(int k=0;k<8;k++) s^=lo[k]^hi[k];
  out[blockIdx.x*blockDim.x+threadIdx.x]=s;
}
__global__ void k_add(u64* out, u64 q, int iters) {
  u64 y[8];
  for (int k=0;k<8;k++) y[k] = threadIdx.x*8+k + blockIdx.x;
  for (int it=0; it<iters; ++it) {
    #pragma unroll
    for (int k=0;k<8;k++) { u64 t = y[k] + y[(k+1)&7]; y[k] = t >= q ? t - q : t; }
  }
  u64 s=0; for(int k=0;k<8;k++) s^=y[k];
  out[blockIdx.x*blockDim.x+threadIdx.x]=s;
}
__global__ void k_copy(const ulonglong2* __restrict__ in, ulonglong2* __restrict__ out, size_t n) {
  size_t i = blockIdx.x*(size_t)blockDim.x+threadIdx.x, st = (size_t)gridDim.x*blockDim.x;
  for (; i<n; i+=st) out[i]=in[i];
}
__global__ void k_read(const ulonglong2* __restrict__ in, u64* out, size_t n) {
  size_t i = blockIdx.x*(size_t)blockDim.x+threadIdx.x, st = (size_t)gridDim.x*blockDim.x;
  u64 s=0; for (; i<n; i+=st){ ulonglong2 v=in[i]; s^=v.x^v.y; }
  if (s==0x1234567) out[0]=s;
}
int main(){
  u64* d; CK(hipMalloc(&d, 1<<26));
  hipEvent_t a,b; hipEventCreate(&a); hipEventCreate(&b);
  int blocks=256*8, threads=256, iters=2000; float ms;
  u64 q = 576460752303423489ULL - 0; // placeholder odd
  u64 w = 123456789123ULL, wp = (u64)(((unsigned __int128)w<<64)/q);
  for (int rep=0;rep<2;rep++){
  hipEventRecord(a); k_shoup<<<blocks,threads>>>(d,w,wp,q,iters); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms,a,b);
  double ops = (double)blocks*threads*iters*8; printf("shoup mulmod: %.1f G/s (%.3f ms)\n", ops/ms/1e6, ms);
  hipEventRecord(a); k_mul128<<<blocks,threads>>>(d,w,iters); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms,a,b);
  printf("mul64x64->128 + acc: %.1f G/s\n", ops/ms/1e6);
  hipEventRecord(a); k_add<<<blocks,threads>>>(d,q,iters); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms,a,b);
  printf("addmod: %.1f G/s\n", ops/ms/1e6);
  }
  size_t bytes = (size_t)4<<30; ulonglong2 *x,*y; CK(hipMalloc(&x,bytes)); CK(hipMalloc(&y,bytes));
  hipMemset(x,1,bytes);
  for (int rep=0;rep<3;rep++){
  hipEventRecord(a); k_copy<<<256*16,256>>>(x,y,bytes/16); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms,a,b);
  printf("copy: %.1f GB/s (r+w)\n", 2.0*bytes/ms/1e6);
  hipEventRecord(a); k_read<<<256*16,256>>>(x,d,bytes/16); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms,a,b);
  printf("read: %.1f GB/s\n", 1.0*bytes/ms/1e6);
  }
  return 0;
}
