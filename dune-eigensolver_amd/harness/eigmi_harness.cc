// eigmi_harness.cc -- the reference harness (src/dune-eigensolver.cc) on libeigmi: same INI keys
// (src/dune-eigensolver.ini: [ev] N m maxiter shift regularization tol verbose overlap method
// seed, [mgs] n m n_iter, [parallel] numthreads), same "-key value" command-line overrides
// (Dune::ParameterTreeParser::readOptions), same experiments and printed lines, so the
// reference's experiment scripts (which grep "eval[", "N_M_TOL_..." and "P_n_m_i_...") run
// unchanged.  Experiments (selected by `-run`, default = the one the reference main calls):
//   largest      largest_eigenvalues_convergence_test  (.cc:631-726)
//   smallest     smallest_eigenvalues_convergence_test (.cc:528-628)
//   eigenvalues  eigenvalues_test, method raes | arpack, parallel.numthreads replicas (.cc:448-525)
//   mgs          mgs_performance_test (.cc:164-300): naive / blocked / vectorized(CholQR) MGS
// ARPACK's computeGenSymShiftInvertMinMagnitude is eig_shift_invert_solve, UMFPACK's factorisation
// the host envelope LU; the arpack "iterations" printed are its thick restarts.
//
//   eigmi_harness [-ini FILE] [-run NAME] [-ev.N 64 ...]     (default FILE: dune-eigensolver.ini)
//   eigmi_harness -print-config ...                          (parse only; no device needed)
#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <map>
#include <mutex>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "eigmi.h"

namespace {

// ------------------------------------------------------------------ ParameterTree stand-in
struct Params {
  std::map<std::string, std::string> kv;
  static std::string trim(const std::string &s)
  {
    const auto a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
    return a == std::string::npos ? "" : s.substr(a, b - a + 1);
  }
  bool read_ini(const std::string &path)
  {
    std::ifstream f(path);
    if (!f) return false;
    std::string line, sec;
    while (std::getline(f, line))
    {
      const auto h = line.find('#');
      if (h != std::string::npos) line = line.substr(0, h);
      line = trim(line);
      if (line.empty()) continue;
      if (line.front() == '[' && line.back() == ']')
      {
        sec = trim(line.substr(1, line.size() - 2));
        continue;
      }
      const auto eq = line.find('=');
      if (eq == std::string::npos) continue;
      const std::string k = trim(line.substr(0, eq)), v = trim(line.substr(eq + 1));
      kv[sec.empty() ? k : sec + "." + k] = v;
    }
    return true;
  }
  // "-key value" pairs, like ParameterTreeParser::readOptions
  void read_options(int argc, char **argv)
  {
    for (int i = 1; i < argc; ++i)
    {
      std::string a = argv[i];
      if (a.size() > 1 && a[0] == '-' && i + 1 < argc && a != "-print-config") kv[a.substr(1)] = argv[++i];
    }
  }
  std::string get(const std::string &k) const
  {
    auto it = kv.find(k);
    if (it == kv.end())
    {
      std::cerr << "missing parameter " << k << std::endl;
      std::exit(2);
    }
    return it->second;
  }
  std::string get(const std::string &k, const std::string &def) const
  {
    auto it = kv.find(k);
    return it == kv.end() ? def : it->second;
  }
  int geti(const std::string &k) const { return std::stoi(get(k)); }
  double getd(const std::string &k) const { return std::stod(get(k)); }
};

void ck(int rc, eig_ctx_t ctx, const char *what)
{
  if (rc == EIG_OK) return;
  std::cerr << what << " failed (" << rc << "): " << eig_last_error(ctx) << std::endl;
  std::exit(3);
}

// the reference's Barrier (.cc:42-89), condition-variable form
class Barrier {
 public:
  explicit Barrier(int P) : P_(P) {}
  int nthreads() const { return P_; }
  void wait()
  {
    if (P_ == 1) return;
    std::unique_lock<std::mutex> l(m_);
    const unsigned long g = gen_;
    if (++count_ == P_)
    {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
    }
    else
      cv_.wait(l, [&] { return gen_ != g; });
  }

 private:
  int P_, count_ = 0;
  unsigned long gen_ = 0;
  std::mutex m_;
  std::condition_variable cv_;
};

struct Timer {
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  void reset() { t0 = std::chrono::steady_clock::now(); }
  double elapsed() const { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); }
};

// .cc:98-156 generators through eig_gen_matrix (0 Dirichlet, 1 Neumann, 2 PU-masked B, 3 identity)
eig_mat_t make_matrix(eig_ctx_t ctx, int kind, int N, int overlap)
{
  const int64_t n = (int64_t)N * N, nnz = eig_gen_nnzb(kind, N);
  std::vector<int64_t> rp(n + 1);
  std::vector<int32_t> c(nnz);
  std::vector<double> v(nnz);
  ck(eig_gen_matrix(kind, N, overlap, rp.data(), c.data(), v.data()), ctx, "eig_gen_matrix");
  eig_mat_t A = nullptr;
  ck(eig_mat_create_bcsr(ctx, n, n, 1, 1, rp.data(), c.data(), v.data(), &A), ctx, "eig_mat_create_bcsr");
  return A;
}

// .cc:437-446
std::vector<double> eigenvalues_laplace_dirichlet_2d(std::size_t N)
{
  std::vector<double> ev(N * N);
  const double h = 1 / (N + 1.0);
  for (std::size_t i = 0; i < N; ++i)
    for (std::size_t j = 0; j < N; ++j)
      ev[j * N + i] = 4.0 * (std::sin(0.5 * h * (i + 1) * M_PI) * std::sin(0.5 * h * (i + 1) * M_PI) +
                             std::sin(0.5 * h * (j + 1) * M_PI) * std::sin(0.5 * h * (j + 1) * M_PI));
  std::sort(ev.begin(), ev.end());
  return ev;
}

// computeGenSymShiftInvertMinMagnitude(B, eps, x, lambda, sigma); returns the "iteration count"
int arpack(eig_ctx_t ctx, eig_mat_t A, eig_mat_t B, double eps, int nev, double sigma, std::vector<double> &lambda)
{
  int restarts = 0;
  lambda.assign(nev, 0.0);
  ck(eig_shift_invert_solve(A, B, nullptr, sigma, nev, 0, eps, 0, 123, lambda.data(), nullptr, &restarts), ctx,
     "computeGenSymShiftInvertMinMagnitude");
  return restarts + 1;
}

// ------------------------------------------------------------------ experiments
int largest_eigenvalues_convergence_test(const Params &pt)
{
  eig_ctx_t ctx;
  ck(eig_ctx_create(0, &ctx), nullptr, "eig_ctx_create");
  const int N = pt.geti("ev.N"), overlap = pt.geti("ev.overlap");
  eig_mat_t A = make_matrix(ctx, 0, N, overlap), B = make_matrix(ctx, 3, N, overlap);
  const int n = N * N, m = pt.geti("ev.m"), maxiter = pt.geti("ev.maxiter");
  const double shift = 0, tol = pt.getd("ev.tol");
  const int verbose = pt.geti("ev.verbose");
  const unsigned seed = (unsigned)std::stoul(pt.get("ev.seed"));
  std::vector<double> eigenvalues_arpack, eigenvalues_arpack2;
  arpack(ctx, A, B, 1e-14, m, -shift, eigenvalues_arpack);
  Timer timer_arpack;
  const int arpackIterations = arpack(ctx, A, B, tol, m, -shift, eigenvalues_arpack2);
  const double time_arpack = timer_arpack.elapsed();
  std::cout << ": arpack elapsed time " << time_arpack << std::endl;
  double maxerror2 = 0.0;
  for (int i = 0; i < m; i++) maxerror2 = std::max(maxerror2, std::abs(eigenvalues_arpack2[i] - eigenvalues_arpack[i]));
  std::vector<double> eval(m, 0.0);
  Timer timer_eigensolver;
  int iters = 0;
  ck(eig_standard_largest(A, shift, tol, maxiter, m, seed, eval.data(), nullptr, &iters, verbose), ctx,
     "StandardLargest");
  const double time_eigensolver = timer_eigensolver.elapsed();
  // the reference calls eigenvalues_laplace_dirichlet_2d(m) (.cc:683: N = m, kept as is)
  std::vector<double> eigenvalues_analytical = eigenvalues_laplace_dirichlet_2d(m);
  double maxerror3 = 0.0;
  for (int i = 0; i < m; ++i) maxerror3 = std::max(maxerror3, std::abs(eval[i] - eigenvalues_analytical[i]));
  std::cout << "eval_num__EIGENSOLVER_ANALYTICAL_ARPACKACR_ARPACKTOL_ESANERROR_ESARERR" << std::endl;
  for (int i = 0; i < (int)eval.size(); i++)
    std::cout << "eval[" << std::setw(3) << i << "]=" << std::setw(10) << std::scientific << std::showpoint
              << std::setprecision(2) << eval[i] << "  " << eigenvalues_analytical[i] << "  " << eigenvalues_arpack[i]
              << "  " << eigenvalues_arpack2[i] << "  " << std::abs(eval[i] - eigenvalues_analytical[i]) << "  "
              << std::abs(eval[i] - eigenvalues_arpack[i]) << std::endl;
  std::cout << ": eigensolver elapsed time " << time_eigensolver << std::endl;
  double maxerror = 0.0;
  for (int i = 0; i < (int)eval.size(); i++) maxerror = std::max(maxerror, std::abs(eval[i] - eigenvalues_arpack[i]));
  std::cout << "N_M_TOL_ESARERROR_ARPERROR_ESANERROR_TIMERATIO_ARPACKITER " << std::endl;
  std::cout << n << " & " << m << " & " << tol << " & " << maxerror << " & " << maxerror2 << " & " << maxerror3
            << " & " << time_eigensolver / time_arpack << " & " << arpackIterations << " \\\\" << std::endl;
  std::cout << "eigmi: StandardLargest iterations " << iters << std::endl;
  eig_mat_destroy(A);
  eig_mat_destroy(B);
  eig_ctx_destroy(ctx);
  return 0;
}

int smallest_eigenvalues_convergence_test(const Params &pt)
{
  eig_ctx_t ctx;
  ck(eig_ctx_create(0, &ctx), nullptr, "eig_ctx_create");
  const int N = pt.geti("ev.N"), overlap = pt.geti("ev.overlap");
  eig_mat_t A = make_matrix(ctx, 1, N, overlap), B = make_matrix(ctx, 2, N, overlap);
  const int n = N * N, m = pt.geti("ev.m"), maxiter = pt.geti("ev.maxiter");
  const double shift = pt.getd("ev.shift"), regularization = pt.getd("ev.regularization"), tol = pt.getd("ev.tol");
  const int verbose = pt.geti("ev.verbose");
  const unsigned seed = (unsigned)std::stoul(pt.get("ev.seed"));
  std::vector<double> eigenvalues_arpack, eigenvalues_arpack2;
  arpack(ctx, A, B, 1e-14, m, -shift, eigenvalues_arpack);
  Timer timer_arpack;
  const int arpackIterations = arpack(ctx, A, B, tol, m, -shift, eigenvalues_arpack2);
  const double time_arpack = timer_arpack.elapsed();
  std::cout << ": arpack elapsed time " << time_arpack << std::endl;
  double maxerror2 = 0.0;
  for (int i = 0; i < m; i++) maxerror2 = std::max(maxerror2, std::abs(eigenvalues_arpack2[i] - eigenvalues_arpack[i]));
  std::vector<double> eval(m);
  Timer timer_eigensolver;
  int iters = 0;
  ck(eig_generalized_inverse(A, B, nullptr, shift, regularization, tol, maxiter, m, seed, eval.data(), nullptr, &iters,
                             verbose),
     ctx, "GeneralizedInverse");
  const double time_eigensolver = timer_eigensolver.elapsed();
  for (int i = 0; i < (int)eval.size(); i++)
    std::cout << "eval[" << std::setw(3) << i << "]=" << std::setw(10) << std::scientific << std::showpoint
              << std::setprecision(2) << eval[i] << " " << std::abs(eval[i] - eigenvalues_arpack2[i]) << std::endl;
  std::cout << ": eigensolver elapsed time " << time_eigensolver << std::endl;
  double maxerror = 0.0;
  for (int i = 0; i < (int)eval.size(); i++) maxerror = std::max(maxerror, std::abs(eval[i] - eigenvalues_arpack2[i]));
  std::cout << "N_M_TOL_RASERROR_ARPERROR_TIMERATIO_ARPACKITER " << n << " & " << m << " & " << tol << " & "
            << maxerror << " & " << maxerror2 << " & " << time_eigensolver / time_arpack << " & " << arpackIterations
            << " \\\\" << std::endl;
  std::cout << "eigmi: GeneralizedInverse iterations " << iters << std::endl;
  eig_mat_destroy(A);
  eig_mat_destroy(B);
  eig_ctx_destroy(ctx);
  return 0;
}

int eigenvalues_test(const Params &pt, int rank, Barrier *pbarrier, int device)
{
  eig_ctx_t ctx;
  ck(eig_ctx_create(device, &ctx), nullptr, "eig_ctx_create");
  const int N = pt.geti("ev.N"), overlap = pt.geti("ev.overlap");
  eig_mat_t A = make_matrix(ctx, 1, N, overlap), B = make_matrix(ctx, 2, N, overlap);
  const int m = pt.geti("ev.m"), maxiter = pt.geti("ev.maxiter");
  const double shift = pt.getd("ev.shift"), regularization = pt.getd("ev.regularization"), tol = pt.getd("ev.tol");
  const int verbose = pt.geti("ev.verbose");
  const std::string method = pt.get("ev.method");
  if (method == "raes")
  {
    std::vector<double> eval(m);
    Timer timer;
    pbarrier->wait();
    timer.reset();
    int iters = 0;
    ck(eig_generalized_inverse(A, B, nullptr, shift, regularization, tol, maxiter, m, 123, eval.data(), nullptr,
                               &iters, verbose),
       ctx, "GeneralizedInverse");
    pbarrier->wait();
    const double time = timer.elapsed();
    if (rank == 0)
    {
      for (int i = 0; i < (int)eval.size(); i++)
        std::cout << "eval[" << std::setw(3) << i << "]=" << std::setw(20) << std::scientific << std::showpoint
                  << std::setprecision(12) << eval[i] << std::endl;
      std::cout << rank << ": eigensolver elapsed time " << time << std::endl;
    }
  }
  if (method == "arpack" && rank == 0)
  {
    std::vector<double> eigenvalues;
    Timer timer;
    arpack(ctx, A, B, tol, m, -shift, eigenvalues);
    const double time = timer.elapsed();
    for (int i = 0; i < (int)eigenvalues.size(); i++)
      std::cout << "eval[" << std::setw(3) << i << "]=" << std::setw(20) << std::scientific << std::showpoint
                << std::setprecision(12) << eigenvalues[i] << std::endl;
    std::cout << rank << ": arpack elapsed time " << time << std::endl;
  }
  eig_mat_destroy(A);
  eig_mat_destroy(B);
  eig_ctx_destroy(ctx);
  return 0;
}

void mgs_performance_test(const Params &pt, int rank, Barrier *pbarrier, int device)
{
  std::cout << "MGS STARTS HERE" << std::endl;
  const std::size_t n = std::stoul(pt.get("mgs.n")), m = std::stoul(pt.get("mgs.m")),
                    n_iter = std::stoul(pt.get("mgs.n_iter"));
  const std::size_t b = 8;
  if (rank == 0)
  {
    std::cout << "n=" << n << std::endl;
    std::cout << "m=" << m << std::endl;
    std::cout << "b=" << b << std::endl;
    std::cout << "n_iter=" << n_iter << std::endl;
  }
  eig_ctx_t ctx;
  ck(eig_ctx_create(device, &ctx), nullptr, "eig_ctx_create");
  double *Q = nullptr;
  ck(eig_malloc(ctx, n * m * 8 + 8, (void **)&Q), ctx, "eig_malloc");
  std::vector<double> h(n * m);
  auto timed = [&](auto fill, auto run) {
    fill();
    ck(eig_memcpy_h2d(ctx, Q, h.data(), n * m * 8), ctx, "upload");
    pbarrier->wait();
    Timer t;
    for (std::size_t iter = 0; iter < n_iter; iter++) run();
    ck(eig_ctx_sync(ctx), ctx, "sync");
    pbarrier->wait();
    return t.elapsed();
  };
  auto fill_cols = [&] {  // MultiVector<double,1>: row-major over (i, j) loops (.cc:190-196)
    std::mt19937 urbg{123};
    std::normal_distribution<double> generator{0.0, 1.0};
    for (std::size_t i = 0; i < n; ++i)
      for (std::size_t j = 0; j < m; ++j) h[j * n + i] = generator(urbg);
  };
  auto fill_blocks = [&] {  // MultiVector<double,8> fill order (.cc:217-221)
    std::mt19937 urbg{123};
    std::normal_distribution<double> generator{0.0, 1.0};
    for (std::size_t bj = 0; bj < m; bj += b)
      for (std::size_t i = 0; i < n; ++i)
        for (std::size_t j = 0; j < b; ++j) h[((bj / 8) * n + i) * 8 + j] = generator(urbg);
  };
  if (rank == 0) std::cout << "start test naive mgs version" << std::endl;
  const double time1 = timed(fill_cols, [&] { ck(eig_orthonormalize_naive(ctx, n, m, Q), ctx, "orthonormalize_naive"); });
  if (rank == 0) std::cout << "start test blocked mgs version" << std::endl;
  const double time2 =
      timed(fill_blocks, [&] { ck(eig_orthonormalize_mv8(ctx, n, m, Q, EIG_ORTHO_MGS), ctx, "orthonormalize_blocked"); });
  if (rank == 0) std::cout << "start test VECTORIZED block mgs version (gfx950 CholQR version)" << std::endl;
  const double time3 = timed(fill_blocks, [&] {
    ck(eig_orthonormalize_mv8(ctx, n, m, Q, EIG_ORTHO_CHOLQR), ctx, "orthonormalize_cholqr");
  });
  if (rank == 0)
  {
    const double P = pbarrier->nthreads();
    const double flops = P * n_iter * eig_flops_orthonormalize(n, m);
    const double bytes = P * n_iter * eig_bytes_orthonormalize_blocked(n, m, (int)b);
    // bytes_orthonormalize_naive (kernels_cpp.hh:108-116)
    double c = 0.0;
    for (std::size_t k = m; k > 0; k--) c += n + 2.0 * n + (k - 1) * (2.0 * n + 3.0 * n);
    const double bytesn = P * n_iter * c * 8;
    std::cout << "P_n_m_i_iblocked_perfn_perfb_perfv " << pbarrier->nthreads() << " " << n << " " << m << " "
              << flops / bytesn << " " << flops / bytes << " " << flops / time1 * 1e-9 << " "
              << flops / time2 * 1e-9 << " " << flops / time3 * 1e-9 << " " << std::endl;
  }
  eig_free(ctx, Q);
  eig_ctx_destroy(ctx);
  std::cout << "MGS ENDS HERE" << std::endl;
}

}  // namespace

int main(int argc, char **argv)
{
  std::cout << "Hello World! This is dune-eigensolver (" << eig_version() << ")." << std::endl;
  Params pt;
  std::string ini = "dune-eigensolver.ini";
  bool print_only = false;
  for (int i = 1; i < argc; ++i)
  {
    if (std::string(argv[i]) == "-ini" && i + 1 < argc) ini = argv[i + 1];
    if (std::string(argv[i]) == "-print-config") print_only = true;
  }
  if (!pt.read_ini(ini)) std::cout << "no ini file " << ini << "; using command-line parameters only" << std::endl;
  pt.read_options(argc, argv);
  if (print_only)
  {
    for (auto &e : pt.kv) std::cout << e.first << " = " << e.second << std::endl;
    return 0;
  }
  const int P = (int)std::thread::hardware_concurrency();
  const int numthreads = std::stoi(pt.get("parallel.numthreads", "1"));
  std::cout << "hardware number of threads is " << P << " number of threads used is " << numthreads << std::endl;
  const std::string run = pt.get("run", "largest");
  int ndev = 0;
  eig_device_count(&ndev);
  if (ndev < 1)
  {
    std::cerr << "no device visible" << std::endl;
    return 4;
  }
  if (run == "largest") return largest_eigenvalues_convergence_test(pt);
  if (run == "smallest") return smallest_eigenvalues_convergence_test(pt);
  if (run == "eigenvalues" || run == "mgs")
  {
    Barrier barrier(numthreads);
    std::vector<std::thread> threads;
    for (int rank = 1; rank < numthreads; ++rank)
      threads.emplace_back([&, rank] {
        if (run == "mgs") mgs_performance_test(pt, rank, &barrier, rank % ndev);
        else eigenvalues_test(pt, rank, &barrier, rank % ndev);
      });
    if (run == "mgs") mgs_performance_test(pt, 0, &barrier, 0);
    else eigenvalues_test(pt, 0, &barrier, 0);
    for (auto &t : threads) t.join();
    return 0;
  }
  std::cerr << "unknown -run " << run << " (largest | smallest | eigenvalues | mgs)" << std::endl;
  return 2;
}
