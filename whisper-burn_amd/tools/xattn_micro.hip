// xattn_micro.hip -- the decode cross-attention kernels (wa_xattn.hip) timed
// in isolation with HIP events, per kernel, at Large-V3 (H = 20, D = 1280,
// T = 1500, Tq = 1, f16x2) and several row counts.  Built by
// scripts/xattn_micro.sh once per WA_XATTN_DIAG attribution variant; the
// numbers are timing only (the inputs are arbitrary, results unchecked).
#include "../csrc/whisper/wa_xattn.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                  \
  do {                                                         \
    hipError_t e = (x);                                        \
    if (e != hipSuccess) {                                     \
      printf("%s failed: %s\n", #x, hipGetErrorString(e));     \
      return 1;                                                \
    }                                                          \
  } while (0)

namespace {
__global__ void fill_half(_Float16* p, size_t n, float amp) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = (_Float16)(amp * (float)((int)((i * 2654435761u) >> 20 & 1023) - 512) / 512.0f);
}
__global__ void fill_float(float* p, size_t n, float amp) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = amp * (float)((int)((i * 2246822519u) >> 19 & 1023) - 512) / 512.0f;
}
// Q4_0 blocks with scale 0.01 and arbitrary nibbles
__global__ void fill_q4(uint8_t* p, size_t nblk) {
  size_t b = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nblk) return;
  uint16_t* h = reinterpret_cast<uint16_t*>(p + b * 18);
  h[0] = __builtin_bit_cast(uint16_t, (_Float16)0.01f);
  for (int i = 1; i < 9; ++i) h[i] = (uint16_t)((b * 40503u + i * 977u) & 0xFFFF);
}
unsigned blocks(size_t n) { return (unsigned)((n + 255) / 256); }
}  // namespace

int main(int argc, char** argv) {
  const int H = 20, D = 1280, T = 1500, NS = 2, HP = 32;
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  std::vector<int> rows = {16, 32, 1, 2, 4, 8};
  const int RMAX = 32;
  _Float16 *enc, *qt, *tiled;
  float *q, *part, *bv;
  uint8_t *wk, *wv;
  const size_t nenc = (size_t)RMAX * T * NS * D;
  CK(hipMalloc(&enc, nenc * 2));
  CK(hipMalloc(&qt, (size_t)RMAX * NS * HP * D * 2));
  CK(hipMalloc(&tiled, (size_t)RMAX * D * 2 * NS + (1 << 20)));
  CK(hipMalloc(&q, (size_t)RMAX * D * 4));
  CK(hipMalloc(&part, wa::xattn_part_floats(RMAX, H, D, T) * 4));
  CK(hipMalloc(&bv, D * 4));
  const size_t wbytes = (size_t)D * (D / 32) * 18;
  CK(hipMalloc(&wk, wbytes));
  CK(hipMalloc(&wv, wbytes));
  hipLaunchKernelGGL(fill_half, dim3(blocks(nenc)), dim3(256), 0, 0, enc, nenc, 2.0f);
  hipLaunchKernelGGL(fill_half, dim3(blocks((size_t)RMAX * NS * HP * D)), dim3(256), 0, 0, qt,
                     (size_t)RMAX * NS * HP * D, 1.0f);
  hipLaunchKernelGGL(fill_float, dim3(blocks((size_t)RMAX * D)), dim3(256), 0, 0, q, (size_t)RMAX * D, 1.0f);
  hipLaunchKernelGGL(fill_float, dim3(blocks(D)), dim3(256), 0, 0, bv, (size_t)D, 0.1f);
  hipLaunchKernelGGL(fill_q4, dim3(blocks(wbytes / 18)), dim3(256), 0, 0, wk, wbytes / 18);
  hipLaunchKernelGGL(fill_q4, dim3(blocks(wbytes / 18)), dim3(256), 0, 0, wv, wbytes / 18);
  uint32_t* wvp;
  CK(hipMalloc(&wvp, wa::wv_pack_words(H, D) * 4));
  CK(wa::launch_wv_pack(wv, H, D, wvp, 0));
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int R : rows) {
    const wa::XattnPlan p = wa::xattn_plan(R, T);
    float* z = part;
    float* ml = part + (size_t)R * p.splits * H * D;
    auto time_it = [&](auto&& launch) -> float {
      for (int i = 0; i < 5; ++i) launch();
      (void)hipEventRecord(a, 0);
      for (int i = 0; i < iters; ++i) launch();
      (void)hipEventRecord(b, 0);
      (void)hipEventSynchronize(b);
      float ms = 0.0f;
      (void)hipEventElapsedTime(&ms, a, b);
      return ms * 1e3f / iters;
    };
    const float t_main = time_it([&] {
      wa::launch_main<1280, 2, 2>(dim3(p.splits, R), qt, enc, 1, T, H, p.splits, p.ch, z, ml, R, 0);
    });
    const float t_q = time_it([&] {
      hipLaunchKernelGGL((wa::xattn_q_mfma_kernel<2, wa::kWtQ4>), dim3(H, D / 64, (R + 31) / 32), dim3(128), 0, 0,
                         q, R, D, wk, HP, qt);
    });
    const float t_out = time_it([&] {
      wa::launch_out<2, wa::kWtQ4>(R, H, z, ml, D, p.splits, wv, wvp, bv, tiled, 0);
    });
    const float t_out4 = time_it([&] {
      wa::launch_out<2, wa::kWtQ4>(R, H, z, ml, D, p.splits, wv, wvp, bv, tiled, 0, true);
    });
    printf("{\"rows\": %d, \"out_split4_us\": %.2f}\n", R, t_out4);
    const float t_all = time_it([&] {
      wa::launch_xattn(q, wk, wv, wvp, bv, wa::kWtQ4, enc, R, 1, T, H, D, qt, part, tiled, NS, 0);
    });
    float t_sc = 0.0f, t_z = 0.0f;
    if (R <= wa::kSmallRowsMax) {  // the split phases one by one
      const int NG = p.splits * p.ch;
      float* sb = part + ((size_t)R * p.splits * H * ((size_t)D + 2) + (size_t)R * H * D + 3) / 4 * 4;
      t_sc = time_it([&] {
        hipLaunchKernelGGL((wa::xattn_scores_kernel<1280, 2, 2, 8>), dim3(NG, R), dim3(512), 0, 0, qt, enc, 1, T, NG, sb);
      });
      t_z = time_it([&] {
        hipLaunchKernelGGL((wa::xattn_z_kernel<1280, 2, 2>), dim3(p.splits, D / 128, R), dim3(256), 0, 0, enc, sb, 1, T,
                           H, p.splits, p.ch, NG, z, ml);
      });
    }
    CK(hipGetLastError());
#if WA_XATTN_STAMP
    {  // phase durations of workgroup (0, 0) in the last timed main launch (clock cycles)
      (void)time_it([&] {
        wa::launch_main<1280, 2, 2>(dim3(p.splits, R), qt, enc, 1, T, H, p.splits, p.ch, z, ml, R, 0);
      });
      unsigned long long st[2][wa::kXsChunks][wa::kXsPhases];
      CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(wa::g_xstamp), sizeof(st)));
      static const char* names[] = {"write_se", "scores", "barrier1", "softmax", "barrier2", "rescale", "z"};
      for (int wv = 0; wv < 2; ++wv) {
        double tot[7] = {0, 0, 0, 0, 0, 0, 0};
        double span = 0;
        const int nch = p.ch;
        for (int c = 0; c < nch && c < wa::kXsChunks; ++c) {
          for (int ph = 0; ph < 7; ++ph) tot[ph] += (double)(st[wv][c][ph + 1] - st[wv][c][ph]);
          span += (double)(st[wv][c][7] - st[wv][c][0]);
        }
        printf("{\"rows\": %d, \"wave\": \"%s\", \"chunks\": %d, \"cycles_per_chunk\": %.0f", R, wv ? "last" : "first",
               nch, span / nch);
        for (int ph = 0; ph < 7; ++ph) printf(", \"%s\": %.0f", names[ph], tot[ph] / nch);
        printf("}\n");
      }
    }
#endif
    printf("{\"rows\": %d, \"scores_us\": %.2f, \"z_us\": %.2f}\n", R, t_sc, t_z);
    const double bytes = (double)R * T * D * 2 * NS;
    printf("{\"small\": %d, \"diag\": %d, \"rows\": %d, \"splits\": %d, \"main_us\": %.2f, \"q_us\": %.2f, \"out_us\": %.2f, "
           "\"all_us\": %.2f, \"main_tbs\": %.3f}\n",
           R <= wa::xattn_small_rows() ? 1 : 0, WA_XATTN_DIAG, R, p.splits, t_main, t_q, t_out, t_all, bytes / (t_main * 1e-6) / 1e12);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
