// ialspp.h -- iALS++ on MI355X (reference ialspp.h:36-553, same public
// surface).
//
// Train() is the reference sequence (ialspp.h:208-251): PredictDataset, then
// per column block [start, start + block_size): the user block Step against
// the items, the item block Step against the new users (Step :351-424 with
// ProjectBlock :85-145), then ComputeLosses / VaR / residual diagnostics.
// Each block Step is one launch of libfrecsys_hip.so (frecsys_pp_step:
// MFMA block SYRK + blocked Cholesky per entity, the prediction vector kept
// on the device); the Gramians come from the same kernels as iALS.
#pragma once

#include <chrono>
#include <cmath>
#include <string>

#include "frecsys/model_base.h"

namespace frecsys {

class IALSppRecommender : public detail::DeviceModel {
 public:
  IALSppRecommender(int embedding_dim, int num_users, int num_items, float reg, float reg_exp,
                    float unobserved_weight, float stdev, float alpha, int block_size,
                    const DeviceOptions& opts = DeviceOptions::FromEnv())
      : DeviceModel(embedding_dim, num_users, num_items, stdev, opts) {
    if (block_size < 1 || block_size > 128)
      LOG(FATAL) << "block_size must be in [1, 128] on the MI355X build (got " << block_size
                 << ")";
    regularization_ = reg;
    regularization_exp_ = reg_exp;
    unobserved_weight_ = unobserved_weight;
    alpha_ = alpha;
    block_size_ = block_size;
    user_loss_ = VectorXf::Zero(num_users);
  }

  VectorXf Score(const int, const SpVector&) override {
    throw("Function 'Score' is not implemented");  // ialspp.h:62-65
  }

  // Fold-in: 8 epochs of block steps from zero user embeddings
  // (ialspp.h:148-206), then GPU scoring + top-K.
  EvaluationResult EvaluateDataset(const VectorXi& k_list, const VectorXf& alpha_list,
                                   const Dataset& data, const SpMatrix& eval_by_user) override {
    std::vector<int32_t> ids;
    Csr csr;
    data.compact_users(&ids, &csr);
    dev_->LoadEval(csr);
    dev_->ZeroEval(dim_);
    const frecsys_solve_params p = params();
    for (int e = 0; e < 8; ++e) {
      dev_->PPPredict(DeviceContext::EVAL);
      for (int start = 0; start < dim_; start += block_size_) {
        const int end = std::min(start + block_size_, dim_);
        dev_->Gramian(DeviceContext::ITEM);
        dev_->PPStep(DeviceContext::EVAL, start, end, p);
      }
    }
    return RankEval(k_list, alpha_list, ids, eval_by_user);
  }

  void Train(const Dataset& data) override {
    dev_->PPLoad(data);
    dev_->PPPredict(DeviceContext::USER);  // ialspp.h:210-216
    const frecsys_solve_params p = params();
    double residual_U = 0, residual_V = 0;
    for (int start = 0; start < dim_; start += block_size_) {  // ialspp.h:220-238
      const int end = std::min(start + block_size_, dim_);
      dev_->Gramian(DeviceContext::ITEM);
      residual_U += dev_->PPStep(DeviceContext::USER, start, end, p);
      dev_->Gramian(DeviceContext::USER);
      residual_V += dev_->PPStep(DeviceContext::ITEM, start, end, p);
    }
    ComputeLosses(data);  // ialspp.h:240
    if (print_varstats_) {  // ialspp.h:241-254
      dev_->Gramian(DeviceContext::ITEM);
      dev_->UserLoss(DeviceContext::USER, unobserved_weight_, false, user_loss_.data());
      PrintVarStats(alpha_);
    }
    if (print_residualstats_)
      LOG(INFO) << format("U residual: {0}, V residual: {1}", (float)std::sqrt(residual_U),
                          (float)std::sqrt(residual_V));
  }

  // ComputeLosses (ialspp.h:258-330), on the GPU parts (frecsys_train_stats).
  void ComputeLosses(const Dataset& data) {
    if (!print_trainstats_) return;
    const auto t0 = std::chrono::steady_clock::now();
    const LossParts lp = ComputeLossParts(data);
    const Csr& uc = data.user_csr();
    const Csr& ic = data.item_csr();
    double loss_reg = 0.0, reg_user_now = 0.0, reg_item_now = 0.0;
    for (int64_t u = 0; u < uc.rows(); ++u) {
      if (!uc.len(u)) continue;
      const double n2 = lp.user_norm2[u];
      loss_reg += n2 * RegularizationValue((int)uc.len(u), (int)num_items_);
      reg_user_now += n2;
    }
    for (int64_t i = 0; i < ic.rows(); ++i) {
      if (!ic.len(i)) continue;
      const double n2 = lp.item_norm2[i];
      loss_reg += n2 * RegularizationValue((int)ic.len(i), (int)num_users_);
      reg_item_now += n2;
    }
    const float loss =
        (float)(lp.observed + unobserved_weight_ * lp.unobserved + loss_reg);
    const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                        std::chrono::steady_clock::now() - t0)
                        .count();
    CheckNaN(loss);
    LOG(INFO) << format(
        "Loss={0:.2f} Loss_observed={1:.2f} Loss_unobserved={2:.2f} Loss_reg={3:.2f} "
        "Loss_reg (user)={4:.2f} Loss_reg (item)={5:.2f}",
        loss, lp.observed / data.num_tuples(), lp.unobserved / num_items_ / num_users_, loss_reg,
        reg_user_now / num_users_, reg_item_now / num_items_);
    LOG(INFO) << format("Time={0}", (int64_t)ms);
  }

  // RegularizationValue (ialspp.h:335-340).
  const float RegularizationValue(int history_size, int num_choices) const {
    return regularization_ *
           std::pow(history_size + unobserved_weight_ * num_choices, regularization_exp_);
  }

 private:
  frecsys_solve_params params() const {
    frecsys_solve_params p = solve_params(FRECSYS_KIND_IALS, regularization_, unobserved_weight_);
    p.reg_exp = regularization_exp_;
    return p;
  }

  float regularization_;
  float regularization_exp_;
  float unobserved_weight_;
  float alpha_;
  int block_size_;
};

}  // namespace frecsys
