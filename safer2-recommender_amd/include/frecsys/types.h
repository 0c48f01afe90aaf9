// types.h -- dense/sparse types of the frecsys public surface.
//
// The reference typedefs Eigen (types.h:23-31): VectorXf, VectorXi, a
// ROW-MAJOR MatrixXf, SpVector = vector<pair<int,int>> (other id, rating
// index) and SpMatrix = unordered_map<int, SpVector>.  Eigen is not a
// dependency here: the embeddings live on the GPU, and the host only needs
// the small subset the CLI, the tests and the evaluation use (construction,
// element access, data(), rows()/size(), mean/min/max, `v << a, b, c`
// comma-initialisation, row views, colwise().mean()).
#pragma once

#include <algorithm>
#include <cassert>
#include <cstdint>
#include <numeric>
#include <unordered_map>
#include <type_traits>
#include <utility>
#include <vector>

namespace frecsys {

namespace detail {

// Eigen 3.4 Redux.h, LinearVectorizedTraversal / NoUnrolling: the sum of a
// plain (packet-accessible, aligned) float vector as the reference's
// -march=native build computes it on an AVX-512 host (Packet16f):
// packet accumulators p0 = x[0:16), p1 = x[16:32), then pairs of packets
// added into p0 and p1 alternately, p0 += p1, one more packet if the aligned
// part has an odd packet count, the horizontal reduction of
// predux<Packet16f> (AVX512DQ: 8 + 8 -> 4 + 4 -> {0+2, 1+3} -> sum), then
// the trailing scalars one by one.  Vectors shorter than one packet sum
// sequentially.  (An AVX2 host would use 8-float packets: the same value up
// to fp32 rounding.)
inline float eigen_packet_sum(const float* x, int64_t n) {
  constexpr int P = 16;
  if (n <= 0) return 0.0f;
  const int64_t aligned = n / P * P, aligned2 = n / (2 * P) * (2 * P);
  if (aligned == 0) {
    float r = x[0];
    for (int64_t i = 1; i < n; ++i) r += x[i];
    return r;
  }
  float p0[P], p1[P];
  for (int k = 0; k < P; ++k) p0[k] = x[k];
  if (aligned > P) {
    for (int k = 0; k < P; ++k) p1[k] = x[P + k];
    for (int64_t i = 2 * P; i < aligned2; i += 2 * P)
      for (int k = 0; k < P; ++k) {
        p0[k] += x[i + k];
        p1[k] += x[i + P + k];
      }
    for (int k = 0; k < P; ++k) p0[k] += p1[k];
    if (aligned > aligned2)
      for (int k = 0; k < P; ++k) p0[k] += x[aligned2 + k];
  }
  float s8[8], s4[4];
  for (int k = 0; k < 8; ++k) s8[k] = p0[k] + p0[k + 8];
  for (int k = 0; k < 4; ++k) s4[k] = s8[k] + s8[k + 4];
  const float t0 = s4[0] + s4[2], t1 = s4[1] + s4[3];
  float r = t0 + t1;
  for (int64_t i = aligned; i < n; ++i) r += x[i];
  return r;
}

}  // namespace detail

template <typename T>
class DenseVector {
 public:
  DenseVector() = default;
  explicit DenseVector(int64_t n) : v_((size_t)std::max<int64_t>(n, 0)) {}
  static DenseVector Zero(int64_t n) { return DenseVector(n); }
  static DenseVector Ones(int64_t n) {
    DenseVector r(n);
    std::fill(r.v_.begin(), r.v_.end(), T(1));
    return r;
  }
  static DenseVector Constant(int64_t n, T x) {
    DenseVector r(n);
    std::fill(r.v_.begin(), r.v_.end(), x);
    return r;
  }
  int64_t size() const { return (int64_t)v_.size(); }
  int64_t rows() const { return size(); }
  T* data() { return v_.data(); }
  const T* data() const { return v_.data(); }
  T& operator()(int64_t i) { return v_[(size_t)i]; }
  const T& operator()(int64_t i) const { return v_[(size_t)i]; }
  T& operator[](int64_t i) { return v_[(size_t)i]; }
  const T& operator[](int64_t i) const { return v_[(size_t)i]; }
  // sum() / mean() restate Eigen's float reductions (detail::eigen_packet_sum
  // below); other element types sum in double.
  T sum() const {
    if constexpr (std::is_same<T, float>::value) {
      return detail::eigen_packet_sum(v_.data(), (int64_t)v_.size());
    } else {
      double s = 0.0;
      for (const T& x : v_) s += (double)x;
      return (T)s;
    }
  }
  // Eigen DenseBase::mean(): sum() / T(size()), in T.
  T mean() const { return v_.empty() ? T(0) : sum() / (T)v_.size(); }
  double sumd() const {
    double s = 0.0;
    for (const T& x : v_) s += (double)x;
    return s;
  }
  T maxCoeff() const { return *std::max_element(v_.begin(), v_.end()); }
  T minCoeff() const { return *std::min_element(v_.begin(), v_.end()); }
  void resize(int64_t n) { v_.resize((size_t)n); }
  std::vector<T>& vec() { return v_; }
  const std::vector<T>& vec() const { return v_; }

  // `k_list << 5, 10, 20;` (Eigen comma initialiser)
  struct CommaInit {
    DenseVector* v;
    int64_t i;
    CommaInit& operator,(T x) {
      assert(i < v->size());
      (*v)(i++) = x;
      return *this;
    }
  };
  CommaInit operator<<(T x) {
    assert(size() > 0);
    (*this)(0) = x;
    return CommaInit{this, 1};
  }

 private:
  std::vector<T> v_;
};

using VectorXf = DenseVector<float>;
using VectorXi = DenseVector<int>;

// Row-major float matrix (types.h:25-27 of the reference).
class MatrixXf {
 public:
  MatrixXf() = default;
  MatrixXf(int64_t rows, int64_t cols) : r_(rows), c_(cols), d_((size_t)(rows * cols)) {}
  static MatrixXf Zero(int64_t rows, int64_t cols) { return MatrixXf(rows, cols); }
  int64_t rows() const { return r_; }
  int64_t cols() const { return c_; }
  int64_t size() const { return r_ * c_; }
  float* data() { return d_.data(); }
  const float* data() const { return d_.data(); }
  float& operator()(int64_t i, int64_t j) { return d_[(size_t)(i * c_ + j)]; }
  float operator()(int64_t i, int64_t j) const { return d_[(size_t)(i * c_ + j)]; }
  float* row(int64_t i) { return d_.data() + i * c_; }
  const float* row(int64_t i) const { return d_.data() + i * c_; }

  struct ColwiseProxy {
    const MatrixXf* m;
    VectorXf mean() const {
      VectorXf out(m->c_);
      for (int64_t j = 0; j < m->c_; ++j) {
        double s = 0.0;
        for (int64_t i = 0; i < m->r_; ++i) s += (*m)(i, j);
        out(j) = m->r_ ? (float)(s / (double)m->r_) : 0.0f;
      }
      return out;
    }
  };
  ColwiseProxy colwise() const { return ColwiseProxy{this}; }

 private:
  int64_t r_ = 0, c_ = 0;
  std::vector<float> d_;
};

// Sparse types (types.h:30-31): (other-side id, rating index) in file order.
using SpVector = std::vector<std::pair<int, int>>;
using SpMatrix = std::unordered_map<int, SpVector>;

}  // namespace frecsys

#ifndef FRECSYS_NO_EIGEN_ALIAS
// The reference's CLI and tests spell the vectors as Eigen::VectorXi /
// Eigen::VectorXf (run_model.cc:32-33); alias them so that code compiles.
namespace Eigen {
using VectorXi = ::frecsys::VectorXi;
using VectorXf = ::frecsys::VectorXf;
}  // namespace Eigen
#endif
