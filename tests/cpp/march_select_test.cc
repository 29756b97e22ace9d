// Host-side unit check of the P1 Kuhn march selection (k_spmv.hip kuhn_variant):
// the value-pack variants 16 / 19 read the pack through one 32-bit buffer descriptor of 64 B per
// row, so a grid with sym_ld * 64 >= 2^31 (2^25 rows and more) must take the band arrays (12).
// No GPU: only the selection function runs.
#include <cstdio>

#include "../../dune-eigensolver_amd/csrc/internal.h"

int main()
{
  int bad = 0;
  auto expect = [&](long long ld, int tune, int want, int gy = 256) {
    eig_mat_s A;
    A.sym_ld = ld;
    A.sym_gy = gy;
    A.tune_march_prefetch = tune;
    const int got = eigmi::kuhn_variant(A);
    if (got != want)
    {
      std::printf("sym_ld %lld tune %d: variant %d, want %d\n", ld, tune, got, want);
      ++bad;
    }
  };
  const long long n256 = 256LL * 256 * 256, n448 = 448LL * 448 * 448, nwrap = 256LL * 512 * 512;
  expect(n256, 0, 20);       // the pack with the line exchange in LDS (lines in groups of 4)
  expect(n256, 0, 16, 254);  // lines not a multiple of 4: the pack alone
  expect(n256, 13, 16);
  expect(n256, 15, 19);
  expect(n256, 14, 12);
  expect((1LL << 25) - 1, 0, 20);
  expect(1LL << 25, 0, 12);  // 64 B * 2^25 = 2^31: the descriptor's record count no longer fits
  expect(n448, 0, 12);
  expect(n448, 15, 12);
  expect(nwrap, 0, 12);      // 64 * 2^26 = 2^32: would wrap to a zero-sized descriptor
  std::printf(bad ? "FAILED\n" : "ALL OK\n");
  return bad ? 1 : 0;
}
