// loopback_test.cc -- the distributed device path on ONE GPU: P virtual ranks (host threads, one
// context each) over libeigmi's in-process loopback transport.  Exercises the row-partitioned
// SELL image with window-local columns, the halo plan, the interior / boundary slice split, the
// split-K1 carry and the allreduce placement of the Lanczos drivers; only the RCCL calls
// themselves are replaced.  Compared with the single-rank run of the same matrix; the generalised
// block Lanczos (config C5, P1 K/M, block 16) likewise, Ritz values to 1e-10 relative.
//
//   loopback_test P N     (defaults 3, 24)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "eigmi.h"

#define CK(x)                                                                               \
  do {                                                                                      \
    int rc_ = (x);                                                                          \
    if (rc_ != EIG_OK) {                                                                    \
      std::printf("FAIL %s -> %d (%s)\n", #x, rc_, eig_last_error(nullptr));                 \
      std::exit(3);                                                                         \
    }                                                                                       \
  } while (0)

struct Rows {
  std::vector<int64_t> rp;
  std::vector<int32_t> c;
  std::vector<double> v;
};

static Rows gen(int N, int64_t b, int64_t cnt, int kind = 4)
{
  Rows r;
  int64_t nnz = eig_gen_nnzb_rows(kind, N, b, cnt);
  r.rp.resize(cnt + 1);
  r.c.resize(nnz > 0 ? nnz : 1);
  r.v.resize(nnz > 0 ? nnz : 1);
  CK(eig_gen_matrix_rows(kind, N, b, cnt, r.rp.data(), r.c.data(), r.v.data()));
  return r;
}

// Generalised block Lanczos (config C5) on the P1 pencil: Ritz values of `bsteps` steps, block 16 on
// the constant-coefficient K / M (kinds 6 / 7); block 32 -- C5's k -- on the variable-coefficient
// pencil (kinds 9 / 10, one coefficient per tetrahedron) when var is set.
static const int kBlk = 16, kBsteps = 6, kBnev = 4;
static void block_lanczos(eig_ctx_t ctx, int N, int64_t b, int64_t cnt, bool dist, double *ev, bool var = false)
{
  const int64_t n = (int64_t)N * N * N;
  Rows k = gen(N, b, cnt, var ? 9 : 6), m = gen(N, b, cnt, var ? 10 : 7);
  eig_mat_t K, M;
  if (dist)
  {
    CK(eig_mat_create_bcsr_dist(ctx, n, b, cnt, 1, 1, k.rp.data(), k.c.data(), k.v.data(), &K));
    CK(eig_mat_create_bcsr_dist(ctx, n, b, cnt, 1, 1, m.rp.data(), m.c.data(), m.v.data(), &M));
  }
  else
  {
    CK(eig_mat_create_bcsr(ctx, n, n, 1, 1, k.rp.data(), k.c.data(), k.v.data(), &K));
    CK(eig_mat_create_bcsr(ctx, n, n, 1, 1, m.rp.data(), m.c.data(), m.v.data(), &M));
  }
  eig_blanczos_t bl;
  CK(eig_blanczos_create(K, M, var ? 32 : kBlk, kBsteps, 36, 0.5, 2.5, 123, &bl));
  CK(eig_blanczos_step(bl, kBsteps, nullptr));
  CK(eig_blanczos_ritz(bl, kBnev, EIG_WHICH_LA, ev, nullptr, nullptr));
  CK(eig_blanczos_destroy(bl));
  eig_mat_destroy(K);
  eig_mat_destroy(M);
}

// Guarded fused step with repairs (k_spmv.hip fused_begin): Poisson plus +100 on the diagonal of
// 12 rows puts trace/n away from the bulk, so some launches repair instead of stepping; the
// repair and the step after it run through the interior / boundary split with the carry.
static const int kRsteps = 14;
static void outliers(int N, int64_t b, Rows &r)
{
  const int64_t n = (int64_t)N * N * N, every = n / 12;
  for (int64_t i = 0; i + 1 < (int64_t)r.rp.size(); ++i)
    for (int64_t p = r.rp[i]; p < r.rp[i + 1]; ++p)
      if (r.c[p] == b + i && (b + i) % every == 0) r.v[p] += 100.0;
}
static void fused_repair_run(eig_mat_t A, double *a, double *be, int *launches, int kind = EIG_LANCZOS_FUSED)
{
  eig_lanczos_t ws;
  CK(eig_lanczos_create_ex(A, kRsteps, nullptr, 123, kind, &ws));
  CK(eig_lanczos_step(ws, kRsteps, 0, nullptr));
  CK(eig_lanczos_tridiag(ws, nullptr, a, be));
  int k = 0;
  CK(eig_lanczos_info(ws, &k, launches));
  CK(eig_lanczos_destroy(ws));
}

// Value-streaming images (k_spmv.hip march variant 15 where the grid allows) and the uniform-
// band check across rank interfaces: (a) the variable-coefficient 7-point matrix (eig_gen kind 8);
// (b) the Poisson matrix whose z couplings across plane pz (rows of planes pz - 1 / pz, both mirror
// entries) are -2: every rank's own upper entries are still one constant per diagonal, but the
// lower entries of rank r's first plane that point at its ghost rows are not, so no
// rank may take the uniform march.  SpMV bitwise and the fused recurrence (split and whole halo
// launches) within 1e-12 of the single-rank run.
static void iface(int N, int64_t b, Rows &r, int64_t pz)
{
  const int64_t D = (int64_t)N * N;
  for (int64_t i = 0; i + 1 < (int64_t)r.rp.size(); ++i)
  {
    const int64_t g = b + i;
    for (int64_t p = r.rp[i]; p < r.rp[i + 1]; ++p)
      if ((g / D == pz && r.c[p] == g - D) || (g / D == pz - 1 && r.c[p] == g + D)) r.v[p] = -2.0;
  }
}
struct ValRun {
  std::vector<double> y, fa, fb, wa, wb;
  int64_t variant = -1, uniform = -1;
};
static void value_run(eig_ctx_t ctx, int N, int64_t b, int64_t cnt, bool dist, int kind, int64_t pz,
                      const std::vector<double> &x, int steps, ValRun &o)
{
  const int64_t n = (int64_t)N * N * N;
  Rows r = gen(N, b, cnt, kind);
  if (pz > 0) iface(N, b, r, pz);
  eig_mat_t A;
  if (dist)
    CK(eig_mat_create_bcsr_dist(ctx, n, b, cnt, 1, 1, r.rp.data(), r.c.data(), r.v.data(), &A));
  else
    CK(eig_mat_create_bcsr(ctx, n, n, 1, 1, r.rp.data(), r.c.data(), r.v.data(), &A));
  eig_mat_info info;
  CK(eig_mat_get_info(A, &info));
  o.variant = info.march_variant;
  o.uniform = info.sym_uniform;
  double *dx, *dy;
  CK(eig_malloc(ctx, info.window * 8, (void **)&dx));
  CK(eig_malloc(ctx, info.window * 8, (void **)&dy));
  CK(eig_memset(ctx, dx, 0, info.window * 8));
  CK(eig_memcpy_h2d(ctx, dx + info.own_offset, x.data() + b, cnt * 8));
  CK(eig_mv(A, dx, dy));
  o.y.resize(cnt);
  CK(eig_memcpy_d2h(ctx, o.y.data(), dy + info.own_offset, cnt * 8));
  eig_free(ctx, dx);
  eig_free(ctx, dy);
  o.fa.resize(steps);
  o.fb.resize(steps + 1);
  CK(eig_lanczos_run(A, steps, nullptr, 123, EIG_LANCZOS_FUSED, o.fa.data(), o.fb.data(), nullptr));
  o.wa = o.fa;
  o.wb = o.fb;
  if (dist)
  {
    CK(eig_mat_tune(A, EIG_TUNE_HALO, 1));
    CK(eig_lanczos_run(A, steps, nullptr, 123, EIG_LANCZOS_FUSED, o.wa.data(), o.wb.data(), nullptr));
  }
  eig_mat_destroy(A);
}
static int value_images(int P, int N, const std::vector<double> &x)
{
  const int64_t n = (int64_t)N * N * N;
  const int steps = 25;
  int failures = 0;
  for (int cs = 0; cs < 2; ++cs)
  {
    const int kind = cs == 0 ? 8 : 4;
    const int64_t pz = cs == 0 ? 0 : N / P;  // the first plane of rank 1
    ValRun ser;
    {
      eig_ctx_t ctx;
      CK(eig_ctx_create(0, &ctx));
      value_run(ctx, N, 0, n, false, kind, pz, x, steps, ser);
      eig_ctx_destroy(ctx);
    }
    void *hub;
    CK(eig_loopback_create(P, &hub));
    std::vector<ValRun> out(P);
    std::vector<int64_t> rb(P), rc(P);
    std::vector<std::thread> th;
    for (int r = 0; r < P; ++r)
      th.emplace_back([&, r] {
        eig_ctx_t ctx;
        CK(eig_ctx_create(0, &ctx));
        CK(eig_comm_init_loopback(ctx, hub, r));
        const int64_t p0 = (int64_t)N * r / P, p1 = (int64_t)N * (r + 1) / P;
        rb[r] = p0 * N * N;
        rc[r] = (p1 - p0) * N * N;
        value_run(ctx, N, rb[r], rc[r], true, kind, pz, x, steps, out[r]);
        eig_ctx_destroy(ctx);
      });
    for (auto &t : th) t.join();
    eig_loopback_destroy(hub);
    const char *nm = cs == 0 ? "variable-coefficient" : "interface-coupling";
    if (ser.uniform != 0)
    {
      std::printf("FAIL %s serial: sym_uniform %lld, expected 0\n", nm, (long long)ser.uniform);
      ++failures;
    }
    for (int r = 0; r < P; ++r)
    {
      if (std::memcmp(out[r].y.data(), ser.y.data() + rb[r], rc[r] * 8) != 0)
      {
        std::printf("FAIL %s rank %d: distributed SpMV not bitwise the serial one\n", nm, r);
        ++failures;
      }
      // (b): ranks 0 and 1 hold the modified couplings; uniform ranks further away are fine
      if (cs == 0 ? out[r].uniform != 0 : (r <= 1 && out[r].uniform != 0))
      {
        std::printf("FAIL %s rank %d: sym_uniform %lld, expected 0\n", nm, r, (long long)out[r].uniform);
        ++failures;
      }
      if (cs == 0 && N % 64 == 0 && out[r].variant != 15 && out[r].variant != -1)
      {
        std::printf("FAIL %s rank %d: march variant %lld, expected the value march (15)\n", nm, r,
                    (long long)out[r].variant);
        ++failures;
      }
      for (int j = 0; j < steps; ++j)
        if (std::fabs(out[r].fa[j] - ser.fa[j]) > 1e-12 * std::fabs(ser.fa[j]) ||
            std::fabs(out[r].fb[j + 1] - ser.fb[j + 1]) > 1e-12 * std::fabs(ser.fb[j + 1]) ||
            std::fabs(out[r].wa[j] - ser.fa[j]) > 1e-12 * std::fabs(ser.fa[j]) ||
            std::fabs(out[r].wb[j + 1] - ser.fb[j + 1]) > 1e-12 * std::fabs(ser.fb[j + 1]))
        {
          std::printf("FAIL %s rank %d fused step %d: alpha %.17g/%.17g/%.17g\n", nm, r, j, out[r].fa[j],
                      out[r].wa[j], ser.fa[j]);
          ++failures;
          break;
        }
    }
  }
  return failures;
}

// The fused step's allreduce inside the step kernel (EIG_AR_MAILBOX_STEP, csrc/xch_dev.h) between
// the virtual ranks (eig_comm_loopback_mailbox: their mailboxes are device pointers of this process),
// with the loopback halo: split launches (interior march + boundary slices, the boundary launch
// completing and exchanging the sums) and whole launches, both within 1e-12 of the serial fused run
// (fa / fb), and the repaired recurrence (outlier diagonal) against its serial run.  Skipped with
// EIGMI_LOOPBACK_NO_MAILBOX=1 (the ranks' kernels wait for each other: one hardware queue per stream).
static int mailbox_phase(int P, int N, int steps, const std::vector<double> &fa, const std::vector<double> &fb,
                         const std::vector<double> &ra, const std::vector<double> &rb, int rl,
                         const std::vector<std::vector<double>> &lra, const std::vector<std::vector<double>> &lrb)
{
  if (std::getenv("EIGMI_LOOPBACK_NO_MAILBOX")) return 0;
  const int64_t n = (int64_t)N * N * N;
  void *hub;
  CK(eig_loopback_create(P, &hub));
  std::vector<std::vector<double>> sa(P, std::vector<double>(steps)), sb(P, std::vector<double>(steps + 1)),
      wa(P, std::vector<double>(steps)), wb(P, std::vector<double>(steps + 1)),
      qa(P, std::vector<double>(kRsteps)), qb(P, std::vector<double>(kRsteps + 1));
  std::vector<int> kind(P, -1), errs(P, -1), ql(P, 0);
  std::vector<std::thread> th;
  for (int r = 0; r < P; ++r)
    th.emplace_back([&, r] {
      eig_ctx_t ctx;
      CK(eig_ctx_create(0, &ctx));
      CK(eig_comm_init_loopback(ctx, hub, r));
      CK(eig_comm_loopback_mailbox(ctx));
      CK(eig_comm_select_allreduce(ctx, EIG_AR_MAILBOX_STEP));
      const int64_t p0 = (int64_t)N * r / P, p1 = (int64_t)N * (r + 1) / P;
      const int64_t b = p0 * N * N, cnt = (p1 - p0) * N * N;
      Rows rows = gen(N, b, cnt);
      eig_mat_t A;
      CK(eig_mat_create_bcsr_dist(ctx, n, b, cnt, 1, 1, rows.rp.data(), rows.c.data(), rows.v.data(), &A));
      CK(eig_lanczos_run(A, steps, nullptr, 123, EIG_LANCZOS_FUSED, sa[r].data(), sb[r].data(), nullptr));
      CK(eig_mat_tune(A, EIG_TUNE_HALO, 1));
      CK(eig_lanczos_run(A, steps, nullptr, 123, EIG_LANCZOS_FUSED, wa[r].data(), wb[r].data(), nullptr));
      eig_mat_destroy(A);
      outliers(N, b, rows);
      CK(eig_mat_create_bcsr_dist(ctx, n, b, cnt, 1, 1, rows.rp.data(), rows.c.data(), rows.v.data(), &A));
      fused_repair_run(A, qa[r].data(), qb[r].data(), &ql[r]);
      eig_mat_destroy(A);
      int nr, rk;
      CK(eig_comm_info(ctx, &nr, &rk, &kind[r], &errs[r]));
      eig_ctx_destroy(ctx);
    });
  for (auto &t : th) t.join();
  eig_loopback_destroy(hub);
  int failures = 0;
  for (int r = 0; r < P; ++r)
  {
    if (kind[r] != EIG_AR_MAILBOX_STEP || errs[r] != 0)
    {
      std::printf("FAIL mailbox-step rank %d: allreduce kind %d, timeouts %d\n", r, kind[r], errs[r]);
      ++failures;
    }
    for (int j = 0; j < steps; ++j)
      if (std::fabs(sa[r][j] - fa[j]) > 1e-12 * std::fabs(fa[j]) ||
          std::fabs(sb[r][j + 1] - fb[j + 1]) > 1e-12 * std::fabs(fb[j + 1]) ||
          std::fabs(wa[r][j] - fa[j]) > 1e-12 * std::fabs(fa[j]) ||
          std::fabs(wb[r][j + 1] - fb[j + 1]) > 1e-12 * std::fabs(fb[j + 1]))
      {
        std::printf("FAIL mailbox-step rank %d fused step %d: alpha split %.17g whole %.17g serial %.17g\n", r, j,
                    sa[r][j], wa[r][j], fa[j]);
        ++failures;
        break;
      }
    if (ql[r] != rl)
    {
      std::printf("FAIL mailbox-step rank %d: %d repaired launches vs %d serial\n", r, ql[r], rl);
      ++failures;
    }
    // (the outlier recurrence amplifies rounding: 1e-10 against the serial run, as the loopback check
    // above; and BITWISE the loopback allreduce's run -- both sum the ranks' sums in rank order)
    for (int j = 0; j < kRsteps; ++j)
      if (std::fabs(qa[r][j] - ra[j]) > 1e-10 * std::fabs(ra[j]) ||
          std::fabs(qb[r][j + 1] - rb[j + 1]) > 1e-10 * std::fabs(rb[j + 1]))
      {
        std::printf("FAIL mailbox-step rank %d repaired step %d: alpha %.17g vs %.17g\n", r, j, qa[r][j], ra[j]);
        ++failures;
        break;
      }
    if (std::memcmp(qa[r].data(), lra[r].data(), kRsteps * 8) != 0 ||
        std::memcmp(qb[r].data(), lrb[r].data(), (kRsteps + 1) * 8) != 0)
    {
      std::printf("FAIL mailbox-step rank %d: repaired recurrence not bitwise the loopback allreduce's\n", r);
      ++failures;
    }
  }
  return failures;
}

int main(int argc, char **argv)
{
  const int P = argc > 1 ? std::atoi(argv[1]) : 3;
  const int N = argc > 2 ? std::atoi(argv[2]) : 24;
  const int64_t n = (int64_t)N * N * N;
  const int steps = 30, nev = 3, ncv = 120;
  int failures = 0;

  // ---- serial reference on one context
  std::vector<double> x(n), y_ser(n), a_ser(steps), b_ser(steps + 1), ev_ser(nev), fa_ser(steps), fb_ser(steps + 1);
  std::vector<double> bev_ser(kBnev), vev_ser(kBnev);
  std::vector<double> ra_ser(kRsteps), rb_ser(kRsteps + 1), pra_ser(kRsteps), prb_ser(kRsteps + 1);
  // pipelined step (EIG_LANCZOS_PIPELINED: SpMV on t_{k-1} while the previous allreduce runs)
  std::vector<double> pa_ser(steps), pb_ser(steps + 1);
  std::vector<std::vector<double>> pal(P, std::vector<double>(steps)), pbe(P, std::vector<double>(steps + 1));
  std::vector<std::vector<double>> pral(P, std::vector<double>(kRsteps)), prbe(P, std::vector<double>(kRsteps + 1));
  int prl_ser = 0;
  std::vector<int> prl(P, 0);
  std::vector<std::vector<double>> ral(P, std::vector<double>(kRsteps)), rbe(P, std::vector<double>(kRsteps + 1));
  int rl_ser = 0;
  std::vector<int> rl(P, 0);
  std::vector<std::vector<double>> bev(P, std::vector<double>(kBnev)), vev(P, std::vector<double>(kBnev));
  for (int64_t i = 0; i < n; ++i) x[i] = std::sin(0.37 * i) + 0.01 * (i % 7);
  {
    eig_ctx_t ctx;
    CK(eig_ctx_create(0, &ctx));
    Rows r = gen(N, 0, n);
    eig_mat_t A;
    CK(eig_mat_create_bcsr(ctx, n, n, 1, 1, r.rp.data(), r.c.data(), r.v.data(), &A));
    CK(eig_mv_host(A, x.data(), y_ser.data()));
    CK(eig_lanczos_run(A, steps, nullptr, 123, 0, a_ser.data(), b_ser.data(), nullptr));
    CK(eig_lanczos_run(A, steps, nullptr, 123, EIG_LANCZOS_FUSED, fa_ser.data(), fb_ser.data(), nullptr));
    CK(eig_lanczos_run(A, steps, nullptr, 123, EIG_LANCZOS_PIPELINED, pa_ser.data(), pb_ser.data(), nullptr));
    CK(eig_lanczos_solve(A, nev, ncv, EIG_WHICH_LA, 123, ev_ser.data(), nullptr, nullptr));
    eig_mat_destroy(A);
    outliers(N, 0, r);
    CK(eig_mat_create_bcsr(ctx, n, n, 1, 1, r.rp.data(), r.c.data(), r.v.data(), &A));
    fused_repair_run(A, ra_ser.data(), rb_ser.data(), &rl_ser);
    fused_repair_run(A, pra_ser.data(), prb_ser.data(), &prl_ser, EIG_LANCZOS_PIPELINED);
    eig_mat_destroy(A);
    block_lanczos(ctx, N, 0, n, false, bev_ser.data());
    block_lanczos(ctx, N, 0, n, false, vev_ser.data(), true);
    eig_ctx_destroy(ctx);
  }

  // ---- P virtual ranks
  void *hub;
  CK(eig_loopback_create(P, &hub));
  std::vector<int> graph_ok(P, 0);
  std::vector<std::vector<double>> fal(P, std::vector<double>(steps)), fbe(P, std::vector<double>(steps + 1));
  std::vector<std::vector<double>> y(P), al(P, std::vector<double>(steps)), be(P, std::vector<double>(steps + 1)),
      ev(P, std::vector<double>(nev));
  std::vector<int64_t> rb(P), rc(P), halo(P), uni(P);
  // EIG_TUNE_HALO = 1 (exchange first, one launch): fused and pipelined recurrences
  std::vector<std::vector<double>> wfal(P, std::vector<double>(steps)), wfbe(P, std::vector<double>(steps + 1)),
      wpal(P, std::vector<double>(steps)), wpbe(P, std::vector<double>(steps + 1));
  std::vector<double> dots(P);
  std::vector<std::thread> th;
  for (int r = 0; r < P; ++r)
    th.emplace_back([&, r] {
      eig_ctx_t ctx;
      CK(eig_ctx_create(0, &ctx));
      CK(eig_comm_init_loopback(ctx, hub, r));
      const int64_t planes = N;
      const int64_t p0 = planes * r / P, p1 = planes * (r + 1) / P;
      const int64_t b = p0 * N * N, cnt = (p1 - p0) * N * N;
      rb[r] = b;
      rc[r] = cnt;
      Rows rows = gen(N, b, cnt);
      eig_mat_t A;
      CK(eig_mat_create_bcsr_dist(ctx, n, b, cnt, 1, 1, rows.rp.data(), rows.c.data(), rows.v.data(), &A));
      eig_mat_info info;
      CK(eig_mat_get_info(A, &info));
      halo[r] = info.halo_recv;
      uni[r] = info.sym_uniform;
      // y = A x through window vectors
      double *dx, *dy, *dd;
      CK(eig_malloc(ctx, info.window * 8, (void **)&dx));
      CK(eig_malloc(ctx, info.window * 8, (void **)&dy));
      CK(eig_malloc(ctx, 8, (void **)&dd));
      CK(eig_memset(ctx, dx, 0, info.window * 8));
      CK(eig_memcpy_h2d(ctx, dx + info.own_offset, x.data() + b, cnt * 8));
      CK(eig_mv(A, dx, dy));
      y[r].resize(cnt);
      CK(eig_memcpy_d2h(ctx, y[r].data(), dy + info.own_offset, cnt * 8));
      // global dot of the owned slices
      CK(eig_dot(ctx, cnt, dx + info.own_offset, dx + info.own_offset, dd));
      CK(eig_memcpy_d2h(ctx, &dots[r], dd, 8));
      // Lanczos recurrence and solver
      CK(eig_lanczos_run(A, steps, nullptr, 123, EIG_LANCZOS_TIME_KERNELS, al[r].data(), be[r].data(), nullptr));
      CK(eig_lanczos_run(A, steps, nullptr, 123, EIG_LANCZOS_FUSED, fal[r].data(), fbe[r].data(), nullptr));
      CK(eig_lanczos_run(A, steps, nullptr, 123, EIG_LANCZOS_PIPELINED, pal[r].data(), pbe[r].data(), nullptr));
      CK(eig_mat_tune(A, EIG_TUNE_HALO, 1));
      CK(eig_lanczos_run(A, steps, nullptr, 123, EIG_LANCZOS_FUSED, wfal[r].data(), wfbe[r].data(), nullptr));
      CK(eig_lanczos_run(A, steps, nullptr, 123, EIG_LANCZOS_PIPELINED, wpal[r].data(), wpbe[r].data(), nullptr));
      CK(eig_mat_tune(A, EIG_TUNE_HALO, 0));
      {
        // capture/replay: the loopback transport cannot be captured, replay must take the same steps eagerly
        std::vector<double> ag(steps), bg(steps + 1);
        eig_lanczos_t ws;
        CK(eig_lanczos_create(A, steps, nullptr, 123, &ws));
        int cap = -1;
        CK(eig_lanczos_capture(ws, steps, 0, &cap));
        CK(eig_lanczos_replay(ws, nullptr));
        CK(eig_lanczos_tridiag(ws, nullptr, ag.data(), bg.data()));
        CK(eig_lanczos_destroy(ws));
        graph_ok[r] = cap == 0 && std::memcmp(ag.data(), al[r].data(), steps * 8) == 0 &&
                      std::memcmp(bg.data(), be[r].data(), (steps + 1) * 8) == 0;
      }
      CK(eig_lanczos_solve(A, nev, ncv, EIG_WHICH_LA, 123, ev[r].data(), nullptr, nullptr));
      {
        outliers(N, b, rows);
        eig_mat_t B;
        CK(eig_mat_create_bcsr_dist(ctx, n, b, cnt, 1, 1, rows.rp.data(), rows.c.data(), rows.v.data(), &B));
        fused_repair_run(B, ral[r].data(), rbe[r].data(), &rl[r]);
        fused_repair_run(B, pral[r].data(), prbe[r].data(), &prl[r], EIG_LANCZOS_PIPELINED);
        eig_mat_destroy(B);
      }
      block_lanczos(ctx, N, b, cnt, true, bev[r].data());
      block_lanczos(ctx, N, b, cnt, true, vev[r].data(), true);
      eig_free(ctx, dx);
      eig_free(ctx, dy);
      eig_free(ctx, dd);
      eig_mat_destroy(A);
      eig_ctx_destroy(ctx);
    });
  for (auto &t : th) t.join();
  eig_loopback_destroy(hub);

  double xx = 0.0;
  for (double v : x) xx += v * v;
  for (int r = 0; r < P; ++r)
  {
    if (!graph_ok[r])
    {
      std::printf("FAIL rank %d: capture/replay differs from eig_lanczos_run\n", r);
      ++failures;
    }
    if (std::memcmp(y[r].data(), y_ser.data() + rb[r], rc[r] * 8) != 0)
    {
      std::printf("FAIL rank %d: distributed SpMV not bitwise equal to the serial one\n", r);
      ++failures;
    }
    const int64_t expect_halo = (r > 0 ? N * N : 0) + (r < P - 1 ? N * N : 0);
    if (halo[r] != expect_halo)
    {
      std::printf("FAIL rank %d: halo %ld != %ld\n", r, (long)halo[r], (long)expect_halo);
      ++failures;
    }
    if (std::fabs(dots[r] - xx) > 1e-12 * xx)
    {
      std::printf("FAIL rank %d: global dot %.17g vs %.17g\n", r, dots[r], xx);
      ++failures;
    }
    for (int j = 0; j < steps; ++j)
      if (std::fabs(al[r][j] - a_ser[j]) > 1e-12 * std::fabs(a_ser[j]) ||
          std::fabs(be[r][j + 1] - b_ser[j + 1]) > 1e-12 * std::fabs(b_ser[j + 1]))
      {
        std::printf("FAIL rank %d step %d: alpha %.17g/%.17g beta %.17g/%.17g\n", r, j, al[r][j], a_ser[j],
                    be[r][j + 1], b_ser[j + 1]);
        ++failures;
        break;
      }
    for (int j = 0; j < steps; ++j)
      if (std::fabs(fal[r][j] - fa_ser[j]) > 1e-12 * std::fabs(fa_ser[j]) ||
          std::fabs(fbe[r][j + 1] - fb_ser[j + 1]) > 1e-12 * std::fabs(fb_ser[j + 1]))
      {
        std::printf("FAIL rank %d fused step %d: alpha %.17g/%.17g beta %.17g/%.17g\n", r, j, fal[r][j], fa_ser[j],
                    fbe[r][j + 1], fb_ser[j + 1]);
        ++failures;
        break;
      }
    for (int j = 0; j < steps; ++j)
      if (std::fabs(wfal[r][j] - fa_ser[j]) > 1e-12 * std::fabs(fa_ser[j]) ||
          std::fabs(wfbe[r][j + 1] - fb_ser[j + 1]) > 1e-12 * std::fabs(fb_ser[j + 1]) ||
          std::fabs(wpal[r][j] - pa_ser[j]) > 1e-12 * std::fabs(pa_ser[j]) ||
          std::fabs(wpbe[r][j + 1] - pb_ser[j + 1]) > 1e-12 * std::fabs(pb_ser[j + 1]))
      {
        std::printf("FAIL rank %d whole-launch (EIG_TUNE_HALO) step %d\n", r, j);
        ++failures;
        break;
      }
    for (int j = 0; j < steps; ++j)
      if (std::fabs(pal[r][j] - pa_ser[j]) > 1e-12 * std::fabs(pa_ser[j]) ||
          std::fabs(pbe[r][j + 1] - pb_ser[j + 1]) > 1e-12 * std::fabs(pb_ser[j + 1]) ||
          std::fabs(pa_ser[j] - a_ser[j]) > 1e-11 * std::fabs(a_ser[j]) ||
          std::fabs(pb_ser[j + 1] - b_ser[j + 1]) > 1e-11 * std::fabs(b_ser[j + 1]))
      {
        std::printf("FAIL rank %d pipelined step %d: alpha %.17g/%.17g/%.17g beta %.17g/%.17g/%.17g\n", r, j,
                    pal[r][j], pa_ser[j], a_ser[j], pbe[r][j + 1], pb_ser[j + 1], b_ser[j + 1]);
        ++failures;
        break;
      }
    if (prl[r] != prl_ser || prl_ser <= kRsteps + 1)
    {
      std::printf("FAIL rank %d: pipelined repair run took %d launches, serial %d\n", r, prl[r], prl_ser);
      ++failures;
    }
    for (int j = 0; j < kRsteps; ++j)
      if (std::fabs(pral[r][j] - pra_ser[j]) > 1e-10 * std::fabs(pra_ser[j]) ||
          std::fabs(prbe[r][j + 1] - prb_ser[j + 1]) > 1e-10 * std::fabs(prb_ser[j + 1]))
      {
        std::printf("FAIL rank %d repaired pipelined step %d\n", r, j);
        ++failures;
        break;
      }
    if (rl[r] != rl_ser || rl_ser <= kRsteps + 1)
    {
      std::printf("FAIL rank %d: fused repair run took %d launches, serial %d (%d steps)\n", r, rl[r], rl_ser,
                  kRsteps);
      ++failures;
    }
    for (int j = 0; j < kRsteps; ++j)
      if (std::fabs(ral[r][j] - ra_ser[j]) > 1e-10 * std::fabs(ra_ser[j]) ||
          std::fabs(rbe[r][j + 1] - rb_ser[j + 1]) > 1e-10 * std::fabs(rb_ser[j + 1]))
      {
        std::printf("FAIL rank %d repaired fused step %d: alpha %.17g/%.17g beta %.17g/%.17g\n", r, j, ral[r][j],
                    ra_ser[j], rbe[r][j + 1], rb_ser[j + 1]);
        ++failures;
        break;
      }
    for (int i = 0; i < nev; ++i)
      if (std::fabs(ev[r][i] - ev_ser[i]) > 1e-10)
      {
        std::printf("FAIL rank %d: Ritz %d %.17g vs %.17g\n", r, i, ev[r][i], ev_ser[i]);
        ++failures;
      }
    for (int i = 0; i < kBnev; ++i)
      if (std::fabs(bev[r][i] - bev_ser[i]) > 1e-10 * std::fabs(bev_ser[i]))
      {
        std::printf("FAIL rank %d: block Lanczos Ritz %d %.17g vs %.17g\n", r, i, bev[r][i], bev_ser[i]);
        ++failures;
      }
    for (int i = 0; i < kBnev; ++i)
      if (std::fabs(vev[r][i] - vev_ser[i]) > 1e-10 * std::fabs(vev_ser[i]))
      {
        std::printf("FAIL rank %d: block Lanczos k = 32, variable coefficients, Ritz %d %.17g vs %.17g\n", r, i,
                    vev[r][i], vev_ser[i]);
        ++failures;
      }
  }
  failures += value_images(P, N, x);
  failures += mailbox_phase(P, N, steps, fa_ser, fb_ser, ra_ser, rb_ser, rl_ser, ral, rbe);
  // every rank's slab of whole planes takes the geometric-mask march (global plane coordinates)
  for (int r = 0; r < P; ++r)
    if (uni[r] != 2)
    {
      std::printf("FAIL rank %d: sym_uniform %lld, expected 2 (geometric row masks)\n", r, (long long)uni[r]);
      ++failures;
    }
  std::printf(failures ? "FAILED %d\n" : "ALL OK (P=%d, N=%d)\n", failures ? failures : P, N);
  return failures ? 1 : 0;
}
