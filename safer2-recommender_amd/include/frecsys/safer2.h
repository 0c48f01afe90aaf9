// safer2.h -- SAFER2 on MI355X (reference safer2.h:35-871, same surface).
//
// Train() (safer2.h:266-334): for each primal-dual iteration the dual
// weights omega from the cached losses and xi (host, double math as the
// reference's erfc/exp), StepU (FRECSYS_KIND_WEIGHTED_U against the cached
// item Gramian), StepV (Gramian U^T diag(omega) U, nu = omega/|H_u|,
// FRECSYS_KIND_WEIGHTED_V with the tail quirk), item_gramian_ = V^T V,
// ComputeUserLoss; then xi by smoothed-quantile Newton with Armijo.
#pragma once

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <future>
#include <random>
#include <tuple>
#include <vector>

#include "frecsys/model_base.h"
#include "frecsys/parallel.h"

namespace frecsys {
namespace quantile {

// Kernel helpers, safer2.h:598-647.  Float arguments, double intermediates,
// float results -- the promotions of the source expressions.
inline float gaussian_kernel(const float u, const float h) {
  return (float)(std::pow(2 * M_PI, -0.5) * std::exp(-std::pow((double)(u / h) * M_SQRT1_2, 2)) /
                 h);
}
inline float gaussian_kernel_cdf(const float u, const float h) {
  return (float)(0.5 * std::erfc(-(double)(u / h) * M_SQRT1_2));
}
inline float gaussian_loss(const float u, const float h, const float alpha) {
  const float ell = h * gaussian_kernel(u, h) + (u / h) * (1 - 2 * gaussian_kernel_cdf(-u, h));
  return (float)((double)((h / 2) * ell) + ((double)(1 - alpha) - 0.5) * (double)u);
}
// gaussian_loss with gaussian_kernel(u, h) = k and gaussian_kernel_cdf(-u, h) = c given
inline float gaussian_loss_from(const float u, const float h, const float alpha, const float k,
                                const float c) {
  const float ell = h * k + (u / h) * (1 - 2 * c);
  return (float)((double)((h / 2) * ell) + ((double)(1 - alpha) - 0.5) * (double)u);
}
inline float epanechnikov_kernel(const float u, const float h) {
  const float uh = u / h;
  return (float)((3.0 / 4.0) * (1 - std::pow((double)uh, 2)) * (int)(std::fabs(uh) < 1) / h);
}
inline float epanechnikov_kernel_cdf(const float u, const float h) {
  const float uh = u / h;
  const int in_supp = (int)(std::fabs(uh) <= 1);
  const int pos = (int)(uh > 1);
  return (float)(((std::pow((double)h, -3) / 4.0) *
                  ((3 * (double)u * std::pow((double)h, 2) - std::pow((double)u, 3)) +
                   2 * std::pow((double)h, 3)) *
                  in_supp) +
                 (double)((1 - in_supp) * pos));
}
inline float epanechnikov_loss(const float u, const float h, const float alpha) {
  const float uh = u / h;
  const int in_supp = (int)(std::fabs(uh) <= 1);
  const int pos = (int)(uh > 1);
  const float ell = (float)(((3.0 / 4.0) * std::pow((double)uh, 2) -
                             (1.0 / 8.0) * std::pow((double)uh, 4) + (3.0 / 8.0)) *
                                in_supp +
                            (double)(std::fabs(uh) * pos));
  return (float)((1.0 / 2.0) * h * ell + ((double)(1 - alpha) - 0.5) * (double)u);
}

struct Smoother {
  float alpha, bandwidth;
  bool epan;
  // EvaluateQuantile (safer2.h:652-689): value, gradient, Hessian of the
  // smoothed quantile objective at xi.  r = loss - xi is formed in float,
  // and each `r.unaryExpr(lambda).mean()` is Eigen's reduction of an
  // expression without packet access (Redux.h DefaultTraversal): a
  // sequential float sum from the first element, then / float(n).
  // The per-sample terms are independent and are computed by the host
  // thread pool into scratch arrays; the three sums then run serially in
  // index order, so the result is bit-identical to the serial loop.
  std::tuple<float, float, float> Evaluate(float xi, const float* loss, int64_t n) const {
    tc.resize((size_t)n);
    tk.resize((size_t)n);
    tl.resize((size_t)n);
    ThreadPool::Get().ParallelFor(n, 512, [&](int64_t lo, int64_t hi) {
      for (int64_t i = lo; i < hi; ++i) {
        const float u = loss[i] - xi;
        if (epan) {
          tc[i] = epanechnikov_kernel_cdf(-u, bandwidth);
          tk[i] = epanechnikov_kernel(-u, bandwidth);
          tl[i] = epanechnikov_loss(u, bandwidth, alpha);
        } else {
          // gaussian_loss(u) re-evaluates gaussian_kernel(u) -- equal bit for
          // bit to gaussian_kernel(-u): (-u)/h = -(u/h) exactly and the
          // kernel squares it -- and gaussian_kernel_cdf(-u): each is
          // evaluated once here (one erfc and one exp per sample)
          const float c = gaussian_kernel_cdf(-u, bandwidth);
          const float k = gaussian_kernel(-u, bandwidth);
          tc[i] = c;
          tk[i] = k;
          tl[i] = gaussian_loss_from(u, bandwidth, alpha, k, c);
        }
      }
    });
    float sc = 0, sk = 0, sl = 0;
    for (int64_t i = 0; i < n; ++i) {
      if (i == 0) {
        sc = tc[i];
        sk = tk[i];
        sl = tl[i];
      } else {
        sc += tc[i];
        sk += tk[i];
        sl += tl[i];
      }
    }
    const float fn = (float)n;
    const float grad = (-(1 - alpha) + sc / fn) / alpha;
    const float H = (sk / fn) / alpha;
    const float value = (sl / fn) / alpha;
    return {value, grad, H};
  }
  mutable std::vector<float> tc, tk, tl;  // per-sample scratch
  // ComputeXiDirection (safer2.h:692-712): Newton step with Armijo
  // backtracking (c = 1e-4, <= 32 halvings, gradient at the trial point).
  float Direction(float xi, const float* loss, int64_t n) const {
    auto [f0, g0, H] = Evaluate(xi, loss, n);
    const float d = g0 / H;
    const float c = 1e-4f;
    float gamma = 1.0f;
    float x = xi + gamma * (-d);
    for (int k = 0; k < 32; k++) {
      auto [fx, gx, Hx] = Evaluate(x, loss, n);
      (void)Hx;
      if (fx > f0 + c * gamma * gx * (-d)) {
        gamma *= 0.5f;
        x = xi + gamma * (-d);
      } else {
        break;
      }
    }
    return -gamma * d;
  }
  float Weight(float loss, float xi) const {  // safer2.h:770-776
    const float r = loss - xi;
    return epan ? 1 - epanechnikov_kernel_cdf(-r, bandwidth) : 1 - gaussian_kernel_cdf(-r, bandwidth);
  }
};

}  // namespace quantile

class SAFER2Recommender : public detail::DeviceModel {
 public:
  SAFER2Recommender(int embedding_dim, int num_users, int num_items, float reg,
                    float unobserved_weight, float bandwidth, float alpha, float stdev,
                    int xi_iterations, int pd_iterations, bool use_epanechnikov, bool use_snr,
                    float sampling_ratio, bool use_cg, float cg_error_tolerance,
                    int cg_max_iterations, const DeviceOptions& opts = DeviceOptions::FromEnv())
      : DeviceModel(embedding_dim, num_users, num_items, stdev, opts),
        smoother_{alpha, bandwidth, use_epanechnikov} {
    if (use_cg) LOG(FATAL) << "use_cg is not supported by the MI355X solve loop (LLT path only)";
    (void)cg_error_tolerance;
    (void)cg_max_iterations;
    regularization_ = reg;
    unobserved_weight_ = unobserved_weight;
    bandwidth_ = bandwidth;
    alpha_ = alpha;
    use_epanechnikov_ = use_epanechnikov;
    prev_xi_ = 0.0f;
    xi_iterations_ = xi_iterations;
    use_snr_ = use_snr;
    sampling_ratio_ = sampling_ratio;
    pd_iterations_ = pd_iterations;
    snr_rng_.seed(opts.seed >= 0 ? (uint32_t)(opts.seed + 7919) : std::random_device{}());
    dual_weight_ = VectorXf::Constant(num_users, alpha);  // safer2.h:56
    user_loss_ = VectorXf::Zero(num_users);
    user_history_size_ = VectorXf::Zero(num_users);
    item_reg_ = VectorXf::Zero(num_items);
    dev_->Gramian(DeviceContext::ITEM);  // item_gramian_ = V^T V, safer2.h:55
  }

  VectorXf Score(const int, const SpVector&) override {
    throw("Function 'Score' is not implemented");  // safer2.h:79-82
  }

  static const VectorXf ProjectU(const SpVector& user_history, const MatrixXf& item_embeddings,
                                 const MatrixXf& gramian, const float reg,
                                 const float unobserved_weight, const float weight, bool use_cg,
                                 const float = 1e-10, const int = 100) {
    if (use_cg) LOG(FATAL) << "use_cg is not supported";
    return detail::ProjectOnDevice(FRECSYS_KIND_WEIGHTED_U, user_history, item_embeddings,
                                   gramian, reg, unobserved_weight, weight, nullptr);
  }
  static const VectorXf ProjectV(const SpVector& item_history, const MatrixXf& user_embeddings,
                                 const MatrixXf& gramian, const float reg,
                                 const float unobserved_weight, const VectorXf& dual_weight,
                                 bool use_cg, const float = 1e-10, const int = 100) {
    if (use_cg) LOG(FATAL) << "use_cg is not supported";
    return detail::ProjectOnDevice(FRECSYS_KIND_WEIGHTED_V, item_history, user_embeddings,
                                   gramian, reg, unobserved_weight, 1.0f, &dual_weight);
  }

  EvaluationResult EvaluateDataset(const VectorXi& k_list, const VectorXf& alpha_list,
                                   const Dataset& data, const SpMatrix& eval_by_user) override {
    // StepU with omega = 1 and the cached item gramian (safer2.h:246-252)
    return FoldInEvaluate(k_list, alpha_list, data, eval_by_user, u_params(false));
  }

  void Train(const Dataset& data) override {
    // FRECSYS_HOST_PROF (diagnostics): wall ms of each Train() phase on stderr
    static const bool hprof = getenv("FRECSYS_HOST_PROF") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    auto t0 = now();
    StartSnrDraws();  // the sample indices of this epoch's ComputeXi, drawn during the solves
    dev_->LoadTraining(data);
    PrintLosses(data);
    auto t1 = now();
    double tw = 0, tu = 0, tv = 0, tl = 0;
    for (int t = 0; t < pd_iterations_; ++t) {
      auto a = now();
      // residual norms (print_residual_stats): omega, U and V against their
      // values before this iteration's updates (safer2.h:475-489, 550-554,
      // 789-793), computed on the device from snapshots
      VectorXf w_prev;
      if (print_residualstats_) w_prev = dual_weight_;
      ComputeUserWeights(data);                                   // safer2.h:272-273
      const float residual_z = print_residualstats_ ? WeightResidual(dual_weight_, w_prev) : 0.0f;
      auto b = now();
      frecsys_solve_params pu = u_params(true);
      if (print_residualstats_) dev_->Snapshot(DeviceContext::USER);
      dev_->Solve(DeviceContext::USER, pu);                       // safer2.h:277-285
      const float residual_U = print_residualstats_ ? dev_->SnapshotResidual(DeviceContext::USER) : 0.0f;
      auto c = now();
      if (print_residualstats_) dev_->Snapshot(DeviceContext::ITEM);
      StepV(data);                                                // safer2.h:288-290
      const float residual_V = print_residualstats_ ? dev_->SnapshotResidual(DeviceContext::ITEM) : 0.0f;
      auto d = now();
      dev_->Gramian(DeviceContext::ITEM);                         // safer2.h:294-295
      dev_->UserLoss(DeviceContext::USER, unobserved_weight_, true, user_loss_.data());
      tw += ms(a, b);
      tu += ms(b, c);
      tv += ms(c, d);
      tl += ms(d, now());
      VectorXf wl(num_users_);
      ThreadPool::Get().ParallelFor(num_users_, 16384, [&](int64_t lo, int64_t hi) {
        for (int64_t u = lo; u < hi; ++u) wl[u] = dual_weight_[u] * user_loss_[u];
      });
      LOG(INFO) << "Weighted Loss: " << wl.mean();                // safer2.h:300-301
      if (print_varstats_) {
        PrintVarStats(alpha_);
        LOG(INFO) << format("Min: {0:.3f}, Mean: {1:.3f}, Max: {2:.3f}", dual_weight_.minCoeff(),
                            dual_weight_.mean(), dual_weight_.maxCoeff());
      }
      if (print_residualstats_)  // safer2.h:323-328
        LOG(INFO) << format("U residual: {0}, V residual: {1}, z residual: {2}", residual_U,
                            residual_V, residual_z);
    }
    auto x0 = now();
    const float xi = ComputeXi(user_loss_, prev_xi_, xi_iterations_);  // safer2.h:331-333
    LOG(INFO) << "Xi:" << xi;
    prev_xi_ = xi;
    if (hprof)
      fprintf(stderr, "[host-prof] train %.2f ms: load+print %.2f weights %.2f solveU %.2f "
              "stepV %.2f gram+loss %.2f xi %.2f\n", ms(t0, now()), ms(t0, t1), tw, tu, tv, tl,
              ms(x0, now()));
  }

  // Initialize (safer2.h:819-838).
  void Initialize(const Dataset& data) {
    StartSnrDraws();
    dev_->LoadTraining(data);
    dev_->Gramian(DeviceContext::ITEM);
    dev_->UserLoss(DeviceContext::USER, unobserved_weight_, true, user_loss_.data());
    const float prev_xi = user_loss_.mean();
    const float xi = ComputeXi(user_loss_, prev_xi, xi_iterations_);
    LOG(INFO) << "Initial Xi:" << xi;
    prev_xi_ = xi;
    ComputeHistoryStats(data);
  }

  // Smoothed-quantile Newton (safer2.h:716-742); use_snr subsamples
  // N_u * sampling_ratio losses per iteration (seeded when --seed is set).
  float ComputeXi(const VectorXf& user_loss, const float prev_xi, const int nr_iterations) {
    float xi = prev_xi;
    const int64_t n = user_loss.size();
    const int ns = (int)(n * sampling_ratio_);
    std::vector<int> idx;
    if (snr_draws_.valid()) {  // drawn ahead from snr_rng_, the same sequence (joined
      idx = snr_draws_.get();  // before snr_rng_ is touched here)
      if (idx.size() != (size_t)nr_iterations * ns) idx.clear();
    }
    for (int t = 0; t < nr_iterations; ++t) {
      float d;
      if (!use_snr_) {
        d = smoother_.Direction(xi, user_loss.data(), n);
      } else {
        std::vector<float> sample((size_t)ns);
        if (!idx.empty()) {
          for (int j = 0; j < ns; j++) sample[j] = user_loss[idx[(size_t)t * ns + j]];
        } else {
          std::uniform_int_distribution<int> uni(0, (int)n - 1);
          for (int j = 0; j < ns; j++) sample[j] = user_loss[uni(snr_rng_)];
        }
        d = smoother_.Direction(xi, sample.data(), ns);
      }
      xi = xi + d;
    }
    return xi;
  }

  // The SNR sample indices depend only on snr_rng_ (not on the losses): the
  // next ComputeXi's are drawn on a helper thread while this thread drives
  // the GPU half-steps (uniform_int_distribution keeps no state between
  // draws, so one distribution object yields the reference's sequence).
  void StartSnrDraws() {
    if (!use_snr_ || xi_iterations_ <= 0 || snr_draws_.valid()) return;
    const int64_t n = num_users_;
    const int ns = (int)(n * sampling_ratio_);
    const int iters = xi_iterations_;
    snr_draws_ = std::async(std::launch::async, [this, n, ns, iters] {
      std::vector<int> idx((size_t)iters * ns);
      std::uniform_int_distribution<int> uni(0, (int)n - 1);
      for (auto& v : idx) v = uni(snr_rng_);
      return idx;
    });
  }

  float GetMeanWeight() const { return dual_weight_.mean(); }  // safer2.h:815-817
  float xi() const { return prev_xi_; }
  const VectorXf& dual_weight() const { return dual_weight_; }

 protected:
  void OnEmbeddingsSet() override { dev_->Gramian(DeviceContext::ITEM); }

 protected:
  // ComputeUserWeights (safer2.h:745-794): only users with a history.
  void ComputeUserWeights(const Dataset& data) {
    const Csr& uc = data.user_csr();
    const int64_t n = std::min<int64_t>(uc.rows(), num_users_);
    ThreadPool::Get().ParallelFor(n, 4096, [&](int64_t lo, int64_t hi) {
      for (int64_t u = lo; u < hi; ++u)
        if (uc.len(u)) dual_weight_[u] = smoother_.Weight(user_loss_[u], prev_xi_);
    });
  }

  // StepV (safer2.h:493-555).
  void StepV(const Dataset& data) {
    (void)data;
    std::vector<float> nu((size_t)num_users_);
    ThreadPool::Get().ParallelFor(num_users_, 16384, [&](int64_t lo, int64_t hi) {
      for (int64_t u = lo; u < hi; ++u) nu[u] = dual_weight_[u] / user_history_size_[u];
    });
    dev_->Gramian(DeviceContext::USER, dual_weight_.data(), ++weight_epoch_);  // :504-509
    frecsys_solve_params p = solve_params(FRECSYS_KIND_WEIGHTED_V, regularization_,
                                          unobserved_weight_);
    p.alpha = alpha_;
    p.entity_reg = item_reg_.data();
    p.other_weight = nu.data();
    dev_->Solve(DeviceContext::ITEM, p);
  }

  frecsys_solve_params u_params(bool with_weights) const {
    frecsys_solve_params p = solve_params(FRECSYS_KIND_WEIGHTED_U, regularization_,
                                          unobserved_weight_);
    p.entity_weight = with_weights ? dual_weight_.data() : nullptr;
    return p;
  }

  // PrintLosses (safer2.h:337-413), diagnostics only.
  void PrintLosses(const Dataset& data) {
    PrintWeightedLosses(data, regularization_, unobserved_weight_, alpha_);
  }

  quantile::Smoother smoother_;
  float regularization_;
  float unobserved_weight_;
  float bandwidth_;
  float alpha_;
  float prev_xi_;
  bool use_epanechnikov_;
  int xi_iterations_;
  bool use_snr_;
  float sampling_ratio_;
  int pd_iterations_;
  uint64_t weight_epoch_ = 0;
  std::mt19937 snr_rng_;
  std::future<std::vector<int>> snr_draws_;  // ComputeXi's next sample indices
};

}  // namespace frecsys
