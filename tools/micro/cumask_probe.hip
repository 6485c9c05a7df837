// Which (XCD, CU) a CU-masked stream's workgroups land on (hipExtStreamCreateWithCUMask).
// For each mask: 2048 workgroups of 64 threads spin ~20 us each and record HW_REG_XCC_ID and the
// CU / SE fields of HW_REG_HW_ID; prints the distinct (xcc, se, cu) triples used and their count.
// Build: hipcc --offload-arch=gfx950 -O2 cumask_probe.hip -o cumask_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <set>
#include <tuple>
#include <vector>

__global__ void probe(unsigned* out) {
  unsigned hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const long long t0 = clock64();
  while (clock64() - t0 < 40000) {
  }
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
}

static void run(const char* name, const std::vector<unsigned>& mask) {
  hipStream_t s;
  if (mask.empty()) {
    if (hipStreamCreate(&s) != hipSuccess) { printf("stream create failed\n"); exit(1); }
  } else if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
    printf("%s: hipExtStreamCreateWithCUMask failed\n", name);
    return;
  }
  const int G = 2048;
  unsigned* d;
  (void)hipMalloc(&d, G * 8);
  hipLaunchKernelGGL(probe, dim3(G), dim3(64), 0, s, d);
  std::vector<unsigned> h(2 * G);
  (void)hipStreamSynchronize(s);
  (void)hipMemcpy(h.data(), d, G * 8, hipMemcpyDeviceToHost);
  std::set<std::tuple<int, int, int>> cus;
  std::set<int> xccs;
  for (int i = 0; i < G; ++i) {
    const unsigned hw = h[2 * i], xcc = h[2 * i + 1] & 0xF;
    const int cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
    cus.insert(std::make_tuple((int)xcc, se * 2 + sh, cu));
    xccs.insert((int)xcc);
  }
  printf("%-28s CUs used %3zu  XCDs {", name, cus.size());
  for (int x : xccs) printf(" %d", x);
  printf(" }  per XCD:");
  for (int x : xccs) {
    int n = 0;
    for (auto& c : cus) n += std::get<0>(c) == x;
    printf(" %d", n);
  }
  printf("\n");
  (void)hipFree(d);
  (void)hipStreamDestroy(s);
}

int main() {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs %d\n", ncu);
  const int W = (ncu + 31) / 32;
  auto mk = [&](auto pred) {
    std::vector<unsigned> m(W, 0u);
    for (int i = 0; i < ncu; ++i)
      if (pred(i)) m[i / 32] |= 1u << (i % 32);
    return m;
  };
  run("default stream", {});
  run("all bits", mk([](int) { return true; }));
  run("bits 0-31", mk([](int i) { return i < 32; }));
  run("bits 0-63", mk([](int i) { return i < 64; }));
  run("bits i%8==0", mk([](int i) { return i % 8 == 0; }));
  run("bits i%8<2", mk([](int i) { return i % 8 < 2; }));
  run("bits i%8>=2", mk([](int i) { return i % 8 >= 2; }));
  run("bits 0-191", mk([](int i) { return i < 192; }));
  run("bits 192-255", mk([](int i) { return i >= 192; }));
  run("bits i%4==0", mk([](int i) { return i % 4 == 0; }));
  return 0;
}
