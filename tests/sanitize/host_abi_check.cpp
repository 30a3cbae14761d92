// Host-side checks of libdl4ss_hip's C ABI under AddressSanitizer + UBSan (CPU only: built by
// tests/test_host_sanitize_cpu.py from every csrc/*.hip with --cuda-host-only and the sanitizers on
// the host side; no device code, no kernel launch).  It drives the host logic of the entry points:
//   * the recurrence planner (dl4ss_birnn_plan_info / _workspace_bytes / _fwd_xw_supported) over a
//     grid of cells, batches, hidden sizes, precisions and co-residency budgets, with the invariants
//     every launcher relies on (grid within the budget, chunks x rows >= B, groups x units >= H);
//   * the GEMM workspace queries (split-K, grouped) over shape grids;
//   * the argument validation of every compute entry point: invalid shapes / null operands must come
//     back as an error code before any device call.
// Prints "ok" and returns 0; any sanitizer report aborts the process (halt_on_error).
#include <cstdio>
#include <cstdlib>
#include <initializer_list>

#include "../../include/dl4ss_hip.h"

static int g_fail = 0;
#define CHECK(c)                                                            \
  do {                                                                      \
    if (!(c)) {                                                             \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                             \
    }                                                                       \
  } while (0)

static void plans() {
  const int Hs[] = {1, 2, 7, 19, 20, 64, 129, 256, 300, 319, 320, 321, 599, 600, 640, 641, 1000};
  const int Bs[] = {1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 31, 32, 33, 48, 64, 100, 128, 256, 1000};
  const int budgets[] = {30, 120, 240, 480};
  for (int budget : budgets) {
    dl4ss_debug_set_rnn_max_wg(budget);  // every later plan uses it: no device query
    for (int cell = 0; cell < 2; ++cell)
      for (int H : Hs)
        for (int B : Bs) {
          bool any = false;
          for (int prec = 0; prec < 2; ++prec) {
            int info[5] = {-1, -1, -1, -1, -1};
            const int rc = dl4ss_birnn_plan_info(cell, B, H, prec, budget, info);
            if (rc != 0) continue;
            any = true;
            const int BC = info[0], NG = info[1], J = info[2], nchunk = info[3], grid = info[4];
            CHECK(BC >= 1 && BC <= 8 && NG >= 1 && J >= 1 && J <= 20 && nchunk >= 1);
            CHECK(BC * nchunk >= B && BC * (nchunk - 1) < B);
            CHECK(NG * J >= H && (NG - 1) * J < H);
            CHECK(grid == 2 * nchunk * NG && grid <= budget);
          }
          const long long ws = dl4ss_birnn_workspace_bytes(cell, B, H);
          // a fp32 forward that does not fit runs as sub-batches: the workspace query still answers
          CHECK(any ? ws > 0 : ws >= -1);
          for (int Kin : {1, 129, 160, 600, 640, 641})
            CHECK(dl4ss_birnn_fwd_xw_supported(cell, B, 251, H, Kin) == 0 ||
                  dl4ss_birnn_fwd_xw_supported(cell, B, 251, H, Kin) == 1);
        }
  }
  dl4ss_debug_set_rnn_max_wg(0);
  int info[5];
  CHECK(dl4ss_birnn_plan_info(2, 4, 300, 1, 240, info) != 0);    // unknown cell
  CHECK(dl4ss_birnn_plan_info(0, 0, 300, 1, 240, info) != 0);    // empty batch
  CHECK(dl4ss_birnn_plan_info(0, 4, 300, 1, 240, nullptr) != 0); // no output
}

static void gemm_queries() {
  const int Ms[] = {1, 127, 128, 129, 8032, 12345};
  const int Ns[] = {1, 100, 128, 600, 2400, 6450};
  const int Ks[] = {1, 63, 64, 600, 2400, 8032};
  for (int M : Ms)
    for (int N : Ns)
      for (int K : Ks) {
        for (int split : {1, 2, 3, 4, 8}) CHECK(dl4ss_gemm_bf16_gl_ws_bytes(M, N, K, split, 1) >= 0);
        CHECK(dl4ss_colsum_bf16_part_bytes(M, N) >= 0);
      }
}

static void validation() {
  float f = 0.f;
  float* p = &f;  // never dereferenced: every call below must fail its argument checks first
  int st = 0;
  CHECK(dl4ss_stft_fwd(nullptr, 2, 32000, 256, 128, DL4SS_STFT_MAG, nullptr, p, nullptr) != 0);     // no input
  CHECK(dl4ss_stft_fwd(p, 2, 32000, 512, 128, DL4SS_STFT_MAG, nullptr, p, nullptr) != 0);           // n_fft
  CHECK(dl4ss_stft_fwd(p, 2, 32000, 256, 64, DL4SS_STFT_MAG, nullptr, p, nullptr) != 0);            // hop
  CHECK(dl4ss_stft_fwd(p, 2, 100, 256, 128, DL4SS_STFT_MAG, nullptr, p, nullptr) != 0);             // too short
  CHECK(dl4ss_stft_fwd(p, 2, 32000, 256, 128, DL4SS_STFT_COMPLEX, nullptr, nullptr, nullptr) != 0); // no X
  CHECK(dl4ss_stft_fwd(p, 0, 32000, 256, 128, DL4SS_STFT_MAG, nullptr, p, nullptr) == 0);           // empty: no-op
  CHECK(dl4ss_istft(nullptr, 2, 251, 256, 128, 0, p, nullptr) != 0);
  CHECK(dl4ss_istft(p, 2, 1, 256, 128, 0, p, nullptr) != 0);
  CHECK(dl4ss_istft_apply(p, p, 2, 0, 251, 0, 0, p, nullptr) != 0);  // k_per_mix
  CHECK(dl4ss_istft_apply(p, p, 2, 1, 251, 2, 0, p, nullptr) != 0);  // mode
  CHECK(dl4ss_birnn_fwd(0, 2, 4, 10, 300, p, p, p, p, p, p, p, p, 1 << 20, &st, nullptr) != 0);   // precision
  CHECK(dl4ss_birnn_fwd(0, 1, 0, 10, 300, p, p, p, p, p, p, p, p, 1 << 20, &st, nullptr) != 0);   // B
  CHECK(dl4ss_birnn_fwd(0, 1, 4, 10, 300, p, p, p, p, p, p, nullptr, p, 1 << 20, &st, nullptr) != 0);  // LSTM cs
  CHECK(dl4ss_birnn_fwd(0, 1, 4, 10, 300, p, p, p, p, p, p, p, p, 16, &st, nullptr) != 0);        // workspace size
  CHECK(dl4ss_birnn_fwd(0, 1, 4, 10, 4096, p, p, p, p, p, p, p, p, 1 << 30, &st, nullptr) != 0);  // H > 640
  CHECK(dl4ss_gemm_bf16_gl(0, 0, 128, 128, 64, p, 60, p, 128, p, 128, nullptr, 0, 0.f, 1, 1, 0, 0, 0, nullptr, 0,
                           nullptr) != 0);  // lda % 8
}

int main() {
  plans();
  gemm_queries();
  validation();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("ok\n");
  return 0;
}
