// Stand-alone timing harness for the implicit-GEMM conv kernel (k_igemm) on
// U-Net layer shapes, with the kernel's ablation switches, so that main-loop
// changes can be measured without the whole training step.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -Iinclude \
//         tools/igemm_bench.cpp -o build/igemm_bench && build/igemm_bench
// Output: one line per (shape, tile, ablation): average us and TF/s.
#include "../unet-segmentation_amd/csrc/igemm.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

using namespace unet;

#define HC(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                            \
    }                                                                     \
  } while (0)

struct Shape {
  const char* name;
  int n, h, ci, co;
};

template <int BM, int BN, int WM, int WN, int BK, int ABL, int PF = 1>
float run(const IgemmArgs& a, int reps) {
  dim3 grid((a.M + BM - 1) / BM, a.N / BN, 1);
  hipEvent_t e0, e1;
  HC(hipEventCreate(&e0));
  HC(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_igemm<BM, BN, WM, WN, BK, ABL, PF>), grid, dim3(WM * WN * 64), 0, 0, a);
  HC(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((k_igemm<BM, BN, WM, WN, BK, ABL, PF>), grid, dim3(WM * WN * 64), 0, 0, a);
  HC(hipEventRecord(e1, 0));
  HC(hipEventSynchronize(e1));
  float ms = 0;
  HC(hipEventElapsedTime(&ms, e0, e1));
  HC(hipGetLastError());
  HC(hipEventDestroy(e0));
  HC(hipEventDestroy(e1));
  return ms / reps;
}

template <int BM, int BN, int WM, int WN>
void sweep_g(const Shape& s, const IgemmArgs& a, const char* tname) {
  if (a.N % BN) return;
  const double fl = 2.0 * a.M * (double)a.N * a.K;
  hipEvent_t e0, e1;
  HC(hipEventCreate(&e0));
  HC(hipEventCreate(&e1));
  HC((go_igemm_g<BM, BN, WM, WN>(a, 0)));
  HC(hipEventRecord(e0, 0));
  for (int r = 0; r < 5; ++r) HC((go_igemm_g<BM, BN, WM, WN>(a, 0)));
  HC(hipEventRecord(e1, 0));
  HC(hipEventSynchronize(e1));
  float ms = 0;
  HC(hipEventElapsedTime(&ms, e0, e1));
  ms /= 5;
  printf("%-10s %-12s %-10s %9.1f us %7.1f TF/s\n", s.name, tname, "glds", ms * 1e3, fl / (ms * 1e-3) / 1e12);
  fflush(stdout);
}

// max |y_variant - y_reference| over the output (correctness of the glds path)
static float maxdiff(const float* a, const float* b, size_t n) {
  std::vector<float> ha(n), hb(n);
  HC(hipMemcpy(ha.data(), a, n * 4, hipMemcpyDeviceToHost));
  HC(hipMemcpy(hb.data(), b, n * 4, hipMemcpyDeviceToHost));
  float m = 0.f;
  for (size_t i = 0; i < n; ++i) m = std::max(m, std::fabs(ha[i] - hb[i]));
  return m;
}

template <int BM, int BN, int WM, int WN, int BK>
void sweep(const Shape& s, const IgemmArgs& a, const char* tname) {
  if (a.N % BN) return;
  const double fl = 2.0 * a.M * (double)a.N * a.K;
  auto rep = [&](const char* abl, float ms) {
    printf("%-10s %-12s %-10s %9.1f us %7.1f TF/s\n", s.name, tname, abl, ms * 1e3, fl / (ms * 1e-3) / 1e12);
    fflush(stdout);
  };
  rep("full", run<BM, BN, WM, WN, BK, 0>(a, 5));
  rep("noglobal", run<BM, BN, WM, WN, BK, 1>(a, 5));
  rep("stale", run<BM, BN, WM, WN, BK, 512>(a, 5));
  rep("stale-nob", run<BM, BN, WM, WN, BK, 512 | 2>(a, 5));
}

int main() {
  const Shape shapes[] = {
      {"down2.c1", 8, 123, 256, 256},
      {"up3.c1", 8, 166, 128, 128},
      {"inc.c1", 8, 510, 64, 64},
      {"down4.c1", 8, 26, 1024, 1024},
  };
  for (const Shape& s : shapes) {
    const int ho = s.h - 2;
    const size_t xin = (size_t)s.n * s.h * s.h * s.ci, yout = (size_t)s.n * ho * ho * s.co;
    float *x, *w, *y, *sc, *sh, *bias;
    double* stats;
    HC(hipMalloc(&x, xin * 4));
    HC(hipMalloc(&w, (size_t)9 * s.ci * s.co * 4));
    HC(hipMalloc(&y, yout * 4));
    HC(hipMalloc(&sc, s.ci * 4));
    HC(hipMalloc(&sh, s.ci * 4));
    HC(hipMalloc(&bias, s.co * 4));
    HC(hipMalloc(&stats, (size_t)kStatGroups * s.co * 2 * 8));
    std::vector<float> hx(xin);
    for (size_t i = 0; i < xin; ++i) hx[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
    HC(hipMemcpy(x, hx.data(), xin * 4, hipMemcpyHostToDevice));
    std::vector<float> hw((size_t)9 * s.ci * s.co), hs(s.ci), hh(s.ci), hb(s.co, 0.f);
    for (size_t i = 0; i < hw.size(); ++i) hw[i] = (float)((int)((i * 7919u) % 201u) - 100) * 1e-4f;
    for (int c = 0; c < s.ci; ++c) {
      hs[c] = 0.5f + 0.1f * (c % 7);
      hh[c] = 0.1f * (c % 5 - 2);
    }
    HC(hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
    HC(hipMemcpy(sc, hs.data(), s.ci * 4, hipMemcpyHostToDevice));
    HC(hipMemcpy(sh, hh.data(), s.ci * 4, hipMemcpyHostToDevice));
    HC(hipMemcpy(bias, hb.data(), s.co * 4, hipMemcpyHostToDevice));
    HC(hipMemset(stats, 0, (size_t)kStatGroups * s.co * 2 * 8));
    IgemmArgs a;
    Src src;
    src.ptr = x;
    src.H = src.W = s.h;
    src.C = s.ci;
    src.scale = sc;
    src.shift = sh;
    a.a.s[0] = a.a.s[1] = src;
    a.a.Cg = a.a.c_split = s.ci;
    a.a.taps_h = a.a.taps_w = 3;
    a.a.Hg = a.a.Wg = ho;
    a.a.nimg = s.n;
    a.b = w;
    a.M = s.n * ho * ho;
    a.N = s.co;
    a.K = 9 * s.ci;
    a.e.bias = bias;
    a.e.d[0] = Dst{y, ho, ho, s.co, 0, 0};
    a.e.stats = stats;
    // correctness of the glds kernels against the register-staged one
    {
      float* y2;
      HC(hipMalloc(&y2, yout * 4));
      IgemmArgs b = a;
      b.e.stats = nullptr;
      HC((go_igemm<128, 64, 2, 2, 16>(b, 0)));
      b.e.d[0].ptr = y2;
      if (s.co % 128 == 0) {
        HC((go_igemm_g<128, 128, 2, 2>(b, 0)));
        printf("%-10s check 128x128 glds vs reg: max|diff| %.3e\n", s.name, maxdiff(y, y2, yout));
        HC((go_igemm_g<256, 128, 4, 2>(b, 0)));
        printf("%-10s check 256x128 glds vs reg: max|diff| %.3e\n", s.name, maxdiff(y, y2, yout));
        HC((go_igemm_g<64, 128, 2, 2>(b, 0)));
        printf("%-10s check 64x128 glds vs reg: max|diff| %.3e\n", s.name, maxdiff(y, y2, yout));
      }
      HC((go_igemm_g<128, 64, 2, 2>(b, 0)));
      printf("%-10s check 128x64 glds vs reg: max|diff| %.3e\n", s.name, maxdiff(y, y2, yout));
      HC(hipFree(y2));
    }
    sweep<256, 128, 4, 2, 16>(s, a, "256x128x16");
    sweep_g<256, 128, 4, 2>(s, a, "256x128g");
    sweep<128, 128, 2, 2, 16>(s, a, "128x128x16");
    sweep_g<128, 128, 2, 2>(s, a, "128x128g");
    sweep<128, 128, 2, 2, 32>(s, a, "128x128x32");
    sweep<64, 128, 2, 2, 16>(s, a, "64x128x16");
    sweep_g<64, 128, 2, 2>(s, a, "64x128g");
    sweep<128, 64, 2, 2, 16>(s, a, "128x64x16");
    sweep_g<128, 64, 2, 2>(s, a, "128x64g");
    HC(hipFree(x));
    HC(hipFree(w));
    HC(hipFree(y));
    HC(hipFree(sc));
    HC(hipFree(sh));
    HC(hipFree(bias));
    HC(hipFree(stats));
  }
  return 0;
}
