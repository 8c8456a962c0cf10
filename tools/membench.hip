// Microbenchmark: random 8-byte reads / CAS over tables of growing size (HBM, TLB and cache reach).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__device__ inline uint64_t mix64(uint64_t h){h^=h>>33;h*=0xff51afd7ed558ccdull;h^=h>>33;h*=0xc4ceb9fe1a85ec53ull;h^=h>>33;return h;}
__global__ void rnd_read(const uint64_t* t, uint64_t mask, uint64_t n, uint64_t* out){
  uint64_t i=blockIdx.x*(uint64_t)blockDim.x+threadIdx.x; if(i>=n) return;
  uint64_t v=t[mix64(i)&mask]; if(v==12345) out[0]=v; }
__global__ void rnd_cas(unsigned long long* t, uint64_t mask, uint64_t n){
  uint64_t i=blockIdx.x*(uint64_t)blockDim.x+threadIdx.x; if(i>=n) return;
  atomicCAS(&t[mix64(i)&mask], 0ull, i+1); }
__global__ void rnd_add(unsigned long long* t, uint64_t mask, uint64_t n){
  uint64_t i=blockIdx.x*(uint64_t)blockDim.x+threadIdx.x; if(i>=n) return;
  atomicAdd(&t[mix64(i)&mask], 1ull); }
__global__ void seq_cas(unsigned long long* t, uint64_t mask, uint64_t n){
  uint64_t i=blockIdx.x*(uint64_t)blockDim.x+threadIdx.x; if(i>=n) return;
  atomicCAS(&t[i&mask], 0ull, i+1); }
__global__ void grp8_cas(unsigned long long* t, uint64_t mask, uint64_t n){
  uint64_t i=blockIdx.x*(uint64_t)blockDim.x+threadIdx.x; if(i>=n) return;
  atomicCAS(&t[((mix64(i>>3)<<3)|(i&7))&mask], 0ull, i+1); }
__global__ void seq_read(const uint4* t, uint64_t n, uint64_t* out){
  uint64_t i=blockIdx.x*(uint64_t)blockDim.x+threadIdx.x; if(i>=n) return;
  uint4 v=t[i]; if(v.x==12345) out[0]=v.y; }
__global__ void strided_read(const uint4* t, uint64_t n, uint64_t* out){ // lane-per-128B-row
  uint64_t i=blockIdx.x*(uint64_t)blockDim.x+threadIdx.x; if(i>=n) return;
  const uint4* r=t+i*8; uint4 a=r[0],b=r[1],c=r[2],d=r[3],e=r[4],f=r[5],g=r[6],h=r[7];
  uint32_t x=a.x^b.x^c.x^d.x^e.x^f.x^g.x^h.x; if(x==12345) out[0]=x; }
int main(){
  uint64_t maxslots=1ull<<29; unsigned long long* t; hipMalloc(&t,maxslots*8); hipMemset(t,0,maxslots*8);
  uint64_t* out; hipMalloc(&out,8);
  hipEvent_t a,b; hipEventCreate(&a); hipEventCreate(&b); float ms;
  const uint64_t n=10000000;
  for(int lg=17; lg<=29; lg+=2){ uint64_t mask=(1ull<<lg)-1;
    for(int rep=0;rep<2;rep++){
    hipEventRecord(a); rnd_read<<<(n+255)/256,256>>>((const uint64_t*)t,mask,n,out); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms,a,b);
    float r=ms;
    hipEventRecord(a); rnd_cas<<<(n+255)/256,256>>>(t,mask,n); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms,a,b);
    float c=ms;
    hipEventRecord(a); rnd_add<<<(n+255)/256,256>>>(t,mask,n); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms,a,b);
    float ad=ms;
    hipMemset(t,0,maxslots*8);
    hipEventRecord(a); seq_cas<<<(n+255)/256,256>>>(t,mask,n); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms,a,b);
    float sc=ms;
    hipMemset(t,0,maxslots*8);
    hipEventRecord(a); grp8_cas<<<(n+255)/256,256>>>(t,mask,n); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms,a,b);
    if(rep) printf("table %6.0f MB: 10M random reads %.3f ms (%.2f G/s), CAS %.3f ms, add %.3f ms, seq CAS %.3f ms, group-8 CAS %.3f ms\n", (double)(mask+1)*8/1e6, r, n/r/1e6, c, ad, sc, ms);
    hipMemset(t,0,maxslots*8);}
  }
  // sequential 16B/lane reads of 1.28 GB vs lane-strided 128B rows
  uint64_t rows=10000000; uint4* ev; hipMalloc(&ev, rows*128); hipMemset(ev,1,rows*128);
  for(int rep=0;rep<3;rep++){
  hipEventRecord(a); seq_read<<<(rows*8+255)/256,256>>>(ev,rows*8,out); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms,a,b);
  float s=ms;
  hipEventRecord(a); strided_read<<<(rows+255)/256,256>>>(ev,rows,out); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms,a,b);
  if(rep) printf("1.28 GB read: coalesced %.3f ms (%.0f GB/s), lane-per-row %.3f ms (%.0f GB/s)\n", s, rows*128/s/1e6, ms, rows*128/ms/1e6);}
  return 0; }
