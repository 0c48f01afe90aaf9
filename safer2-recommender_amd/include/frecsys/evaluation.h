// evaluation.h -- ranking metrics containers (reference evaluation.h:25-102).
//
// EvaluationResult holds per-user Recall/NDCG at each K; show() logs the
// means ("Mean Rec@K=..." / "Mean NDCG@K=...") and the lower-tail CVaR of
// the per-user metric at each alpha ("Rec CVaR (q=0.10)@5=...").
#pragma once

#include <algorithm>
#include <sstream>
#include <string>
#include <vector>

#include "frecsys/logging.h"
#include "frecsys/types.h"

namespace frecsys {

struct UserEvaluationResult {
  VectorXf recall;
  VectorXf ndcg;
};

struct EvaluationResult {
  VectorXi k_list;
  VectorXf alpha_list;
  MatrixXf recall;  // users x |k_list|
  MatrixXf ndcg;

  // "name@K=value" joined by spaces (evaluation.h:33-47).
  std::string format(const std::string& measure, const VectorXf& m) const {
    std::string out;
    for (int64_t i = 0; i < k_list.size(); ++i) {
      out += ::frecsys::format("{0}@{1}={2:.4f}", measure, k_list[i], m[i]);
      if (i + 1 != k_list.size()) out += " ";
    }
    return out;
  }

  // Mean over the users of column j of `m` (MatrixXf is users x K).
  void show() const {
    LOG(INFO) << format("Mean Rec", recall.colwise().mean());
    LOG(INFO) << format("Mean NDCG", ndcg.colwise().mean());
    const int64_t nk = k_list.size(), na = alpha_list.size();
    std::vector<VectorXf> rec_cvar(na, VectorXf(nk)), ndcg_cvar(na, VectorXf(nk));
    for (int64_t i = 0; i < nk; ++i) {
      VectorXf rc = cvar(column(recall, i)), nc = cvar(column(ndcg, i));
      for (int64_t j = 0; j < na; ++j) {
        rec_cvar[j][i] = rc[j];
        ndcg_cvar[j][i] = nc[j];
      }
    }
    for (int64_t j = 0; j < na; ++j) {
      LOG(INFO) << format(::frecsys::format("Rec CVaR (q={0:.2f})", alpha_list[j]), rec_cvar[j]);
      LOG(INFO) << format(::frecsys::format("NDCG CVaR (q={0:.2f})", alpha_list[j]), ndcg_cvar[j]);
    }
  }

  // Mean of the worst floor(n*alpha)+1 values for each alpha
  // (evaluation.h:83-102: the running mean is taken at sorted position
  // pos = int(n * alpha)).
  VectorXf cvar(const std::vector<float>& m) const {
    std::vector<float> ms(m);
    std::sort(ms.begin(), ms.end());
    VectorXf out = VectorXf::Zero(alpha_list.size());
    int64_t counter = 0;
    float acc = 0.0f;
    for (int64_t i = 0; i < (int64_t)ms.size(); ++i) {
      acc += ms[i];
      for (int64_t j = counter; j < alpha_list.size(); ++j) {
        const int pos = (int)((float)ms.size() * alpha_list[j]);
        if (pos == i) {
          out[counter] = acc / (float)(i + 1);
          counter++;
        }
      }
    }
    return out;
  }

 private:
  static std::vector<float> column(const MatrixXf& m, int64_t j) {
    std::vector<float> c((size_t)m.rows());
    for (int64_t i = 0; i < m.rows(); ++i) c[(size_t)i] = m(i, j);
    return c;
  }
};

}  // namespace frecsys
