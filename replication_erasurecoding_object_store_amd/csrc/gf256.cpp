// gf256.cpp -- see gf256.hpp.
#include "gf256.hpp"

#include <utility>

namespace rs {

const Field& field() {
  static const Field f;
  return f;
}

Matrix multiply(const Matrix& x, const Matrix& y) {
  const Field& F = field();
  Matrix out(x.rows, y.cols);
  for (int r = 0; r < x.rows; ++r)
    for (int c = 0; c < y.cols; ++c) {
      uint8_t acc = 0;
      for (int i = 0; i < x.cols; ++i) acc ^= F.mul(x.at(r, i), y.at(i, c));
      out.at(r, c) = acc;
    }
  return out;
}

// Gauss-Jordan elimination on [A | I]; the inverse is unique, so any pivot order
// yields the bytes the reference's matrix.go Invert yields.
bool invert(const Matrix& in, Matrix* out) {
  const Field& F = field();
  const int n = in.rows;
  Matrix w(n, 2 * n);
  for (int r = 0; r < n; ++r) {
    for (int c = 0; c < n; ++c) w.at(r, c) = in.at(r, c);
    w.at(r, n + r) = 1;
  }
  for (int col = 0; col < n; ++col) {
    int piv = col;
    while (piv < n && w.at(piv, col) == 0) ++piv;
    if (piv == n) return false;
    if (piv != col)
      for (int c = 0; c < 2 * n; ++c) std::swap(w.at(piv, c), w.at(col, c));
    const uint8_t s = F.inv(w.at(col, col));
    for (int c = 0; c < 2 * n; ++c) w.at(col, c) = F.mul(w.at(col, c), s);
    for (int r = 0; r < n; ++r) {
      const uint8_t f = w.at(r, col);
      if (r == col || f == 0) continue;
      for (int c = 0; c < 2 * n; ++c) w.at(r, c) ^= F.mul(f, w.at(col, c));
    }
  }
  *out = Matrix(n, n);
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < n; ++c) out->at(r, c) = w.at(r, n + c);
  return true;
}

Matrix build_encode_matrix(int k, int m) {
  const Field& F = field();
  Matrix v(k + m, k);
  for (int r = 0; r < k + m; ++r)
    for (int c = 0; c < k; ++c) v.at(r, c) = F.pow(static_cast<uint8_t>(r), c);
  Matrix top(k, k);
  for (int r = 0; r < k; ++r)
    for (int c = 0; c < k; ++c) top.at(r, c) = v.at(r, c);
  Matrix top_inv;
  invert(top, &top_inv);  // distinct Vandermonde points: never singular for K+M <= 256
  return multiply(v, top_inv);
}

}  // namespace rs
