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
#include <utility>
#include <vector>

namespace frecsys {

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
  // Sum in double, returned in T (Eigen sums in T with SIMD partials; the
  // double accumulation is the more accurate restatement).
  T sum() const {
    double s = 0.0;
    for (const T& x : v_) s += (double)x;
    return (T)s;
  }
  T mean() const { return v_.empty() ? T(0) : (T)(sumd() / (double)v_.size()); }
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
