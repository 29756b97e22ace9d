// mm.cpp -- Matrix Market import / export.  The reference only generates its
// matrices in memory (src/dune-eigensolver.cc:98-156); real DUNE / PDELab operators reach other
// programs as Matrix Market files written by Dune::storeMatrixMarket (scalar coordinate entries,
// 1-based).  Host-only: the arrays feed eig_mat_create_bcsr / _dist unchanged.
//
// Read: "%%MatrixMarket matrix coordinate {real|integer|pattern} {general|symmetric}"; symmetric
// files are mirrored, duplicate entries summed, columns sorted per row; with br > 1 the scalar
// entries are grouped into br x br blocks (row-major FieldMatrix layout, absent entries 0), which
// is how a BCRSMatrix<FieldMatrix<double,br,br>> is written scalar by scalar.
#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/eigmi.h"

namespace {

typedef int64_t i64;

struct Coo {
  i64 nr = 0, nc = 0;
  std::vector<i64> r, c;
  std::vector<double> v;
};

int read_coo(const char *path, Coo &m)
{
  std::ifstream f(path);
  if (!f) return EIG_ERR_ARG;
  std::string line;
  if (!std::getline(f, line)) return EIG_ERR_ARG;
  std::string lower = line;
  for (auto &ch : lower) ch = (char)std::tolower((unsigned char)ch);
  if (lower.rfind("%%matrixmarket", 0) != 0 || lower.find("matrix") == std::string::npos ||
      lower.find("coordinate") == std::string::npos)
    return EIG_ERR_ARG;
  const bool pattern = lower.find("pattern") != std::string::npos;
  const bool symmetric = lower.find("symmetric") != std::string::npos;
  if (lower.find("complex") != std::string::npos || lower.find("hermitian") != std::string::npos ||
      lower.find("skew") != std::string::npos)
    return EIG_ERR_ARG;
  i64 nnz = -1;
  while (std::getline(f, line))
  {
    if (line.empty() || line[0] == '%') continue;
    std::istringstream is(line);
    if (!(is >> m.nr >> m.nc >> nnz)) return EIG_ERR_ARG;
    break;
  }
  if (nnz < 0 || m.nr < 0 || m.nc < 0) return EIG_ERR_ARG;
  m.r.reserve(symmetric ? 2 * nnz : nnz);
  for (i64 k = 0; k < nnz; ++k)
  {
    i64 i, j;
    double v = 1.0;
    if (!(f >> i >> j)) return EIG_ERR_ARG;
    if (!pattern && !(f >> v)) return EIG_ERR_ARG;
    if (i < 1 || j < 1 || i > m.nr || j > m.nc) return EIG_ERR_SHAPE;
    m.r.push_back(i - 1);
    m.c.push_back(j - 1);
    m.v.push_back(v);
    if (symmetric && i != j)
    {
      m.r.push_back(j - 1);
      m.c.push_back(i - 1);
      m.v.push_back(v);
    }
  }
  return EIG_OK;
}

// CSR (blocked) from the coordinates: per block row, block columns ascending, duplicates summed.
int to_bcsr(const Coo &m, int br, i64 &nbr, i64 &nbc, std::vector<i64> &rp, std::vector<int32_t> &col,
            std::vector<double> &val)
{
  if (br < 1 || br > 4 || m.nr % br || m.nc % br) return EIG_ERR_BLOCKSIZE;
  nbr = m.nr / br;
  nbc = m.nc / br;
  if (nbc >= INT32_MAX) return EIG_ERR_SHAPE;
  std::vector<std::map<i64, std::vector<double>>> rows(nbr);
  for (size_t k = 0; k < m.r.size(); ++k)
  {
    auto &b = rows[m.r[k] / br][m.c[k] / br];
    if (b.empty()) b.assign((size_t)br * br, 0.0);
    b[(m.r[k] % br) * br + (m.c[k] % br)] += m.v[k];
  }
  rp.assign(nbr + 1, 0);
  col.clear();
  val.clear();
  for (i64 i = 0; i < nbr; ++i)
  {
    for (auto &e : rows[i])
    {
      col.push_back((int32_t)e.first);
      val.insert(val.end(), e.second.begin(), e.second.end());
    }
    rp[i + 1] = (i64)col.size();
  }
  return EIG_OK;
}

}  // namespace

extern "C" int eig_mm_read_info(const char *path, int br, int64_t *nb_rows, int64_t *nb_cols, int64_t *nnzb)
{
  if (!path) return EIG_ERR_ARG;
  Coo m;
  int rc = read_coo(path, m);
  if (rc != EIG_OK) return rc;
  i64 nr, nc;
  std::vector<i64> rp;
  std::vector<int32_t> c;
  std::vector<double> v;
  rc = to_bcsr(m, br, nr, nc, rp, c, v);
  if (rc != EIG_OK) return rc;
  if (nb_rows) *nb_rows = nr;
  if (nb_cols) *nb_cols = nc;
  if (nnzb) *nnzb = rp[nr];
  return EIG_OK;
}

extern "C" int eig_mm_read(const char *path, int br, int64_t *rowptr, int32_t *col, double *vals)
{
  if (!path || !rowptr || !col || !vals) return EIG_ERR_ARG;
  Coo m;
  int rc = read_coo(path, m);
  if (rc != EIG_OK) return rc;
  i64 nr, nc;
  std::vector<i64> rp;
  std::vector<int32_t> c;
  std::vector<double> v;
  rc = to_bcsr(m, br, nr, nc, rp, c, v);
  if (rc != EIG_OK) return rc;
  std::copy(rp.begin(), rp.end(), rowptr);
  std::copy(c.begin(), c.end(), col);
  std::copy(v.begin(), v.end(), vals);
  return EIG_OK;
}

extern "C" int eig_mm_write(const char *path, int64_t nb_rows, int64_t nb_cols, int br, int bc, const int64_t *rowptr,
                            const int32_t *col, const double *vals, int symmetric)
{
  if (!path || !rowptr || (rowptr[nb_rows] > 0 && (!col || !vals)) || br < 1 || bc < 1) return EIG_ERR_ARG;
  if (symmetric && (br != bc || nb_rows != nb_cols)) return EIG_ERR_SHAPE;
  std::FILE *f = std::fopen(path, "w");
  if (!f) return EIG_ERR_ARG;
  i64 cnt = 0;
  for (i64 r = 0; r < nb_rows; ++r)
    for (i64 p = rowptr[r]; p < rowptr[r + 1]; ++p)
      for (int a = 0; a < br; ++a)
        for (int b = 0; b < bc; ++b)
        {
          const i64 i = r * br + a, j = (i64)col[p] * bc + b;
          if (!symmetric || j <= i) ++cnt;
        }
  std::fprintf(f, "%%%%MatrixMarket matrix coordinate real %s\n", symmetric ? "symmetric" : "general");
  std::fprintf(f, "%% written by libeigmi (eig_mm_write)\n");
  std::fprintf(f, "%lld %lld %lld\n", (long long)(nb_rows * br), (long long)(nb_cols * bc), (long long)cnt);
  for (i64 r = 0; r < nb_rows; ++r)
    for (i64 p = rowptr[r]; p < rowptr[r + 1]; ++p)
      for (int a = 0; a < br; ++a)
        for (int b = 0; b < bc; ++b)
        {
          const i64 i = r * br + a, j = (i64)col[p] * bc + b;
          if (symmetric && j > i) continue;
          std::fprintf(f, "%lld %lld %.17g\n", (long long)(i + 1), (long long)(j + 1), vals[p * br * bc + a * bc + b]);
        }
  const int ok = std::fclose(f) == 0;
  return ok ? EIG_OK : EIG_ERR_ARG;
}
