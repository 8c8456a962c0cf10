#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <vector>
#include <algorithm>
int run(int lo, int hi, int n) {
  std::vector<unsigned long long> h(n);
  unsigned long long x = 1;
  const unsigned long long kmask = (hi - lo == 64) ? ~0ull : ((1ull << (hi - lo)) - 1);
  for (int i = 0; i < n; i++) { x = x * 6364136223846793005ull + 1442695040888963407ull;
    unsigned long long key = (x >> 20) % 40000 & kmask; unsigned long long other = x * 0x9E3779B97F4A7C15ull;
    unsigned long long fieldmask = kmask << lo; h[i] = (other & ~fieldmask) | (key << lo); }
  unsigned long long *a, *b; (void)hipMalloc(&a, n * 8); (void)hipMalloc(&b, n * 8);
  (void)hipMemcpy(a, h.data(), n * 8, hipMemcpyHostToDevice);
  size_t bytes = 0; (void)hipcub::DeviceRadixSort::SortKeys(nullptr, bytes, a, b, n, lo, hi, 0);
  void* t; (void)hipMalloc(&t, bytes);
  (void)hipcub::DeviceRadixSort::SortKeys(t, bytes, a, b, n, lo, hi, 0);
  std::vector<unsigned long long> o(n); (void)hipMemcpy(o.data(), b, n * 8, hipMemcpyDeviceToHost);
  int bad = 0; for (int i = 1; i < n; i++) if (((o[i] >> lo) & kmask) < ((o[i-1] >> lo) & kmask)) bad++;
  std::sort(h.begin(), h.end()); std::vector<unsigned long long> o2 = o; std::sort(o2.begin(), o2.end());
  printf("bits [%d,%d) n=%d: order violations %d, multiset equal %d\n", lo, hi, n, bad, (int)(o2 == h));
  hipFree(a); hipFree(b); hipFree(t);
  return 0;
}
int main() {
  for (int n : {200000, 20000000}) {
    run(48, 64, n); run(0, 16, n); run(32, 48, n); run(40, 56, n); run(0, 64, n); run(46, 64, n);
  }
  return 0;
}
