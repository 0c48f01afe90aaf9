// recommender.h -- abstract model API (reference recommender.h:37-209).
//
// Keeps the reference's virtual surface (Score, EvaluateDataset, Train,
// SetPrint*Stats) and its evaluation: per held-out user the full score
// vector, history excluded, top-K by nth_element + stable_sort, Recall@K
// and NDCG@K (recommender.h:132-199).  Scoring/top-K runs on host threads
// in this round (SURVEY 8(f) rank 1 -- not part of the solve loop); the
// fold-in solve that precedes it runs on the GPU (model classes).
#pragma once

#include <algorithm>
#include <atomic>
#include <cmath>
#include <limits>
#include <numeric>
#include <random>
#include <set>
#include <thread>
#include <unordered_map>
#include <vector>

#include "frecsys/dataset.h"
#include "frecsys/evaluation.h"
#include "frecsys/logging.h"
#include "frecsys/types.h"

namespace frecsys {

class Recommender {
 public:
  virtual ~Recommender() {}

  virtual VectorXf Score(const int user_id, const SpVector& user_history) {
    (void)user_id;
    (void)user_history;
    return VectorXf::Zero(1);
  }

  virtual EvaluationResult EvaluateDataset(const VectorXi& k_list, const VectorXf& alpha_list,
                                           const Dataset& data, const SpMatrix& eval_by_user) {
    std::unordered_map<int, int> user_to_ind;
    int n = 0;
    for (const auto& kv : eval_by_user) user_to_ind[kv.first] = n++;
    return EvaluateDatasetInternal(
        data.max_item() + 1, k_list, alpha_list, user_to_ind, data, eval_by_user,
        [&](const int user_id, const SpVector& history) { return Score(user_id, history); });
  }

  virtual void Train(const Dataset& dataset) { (void)dataset; }
  virtual void SetPrintTrainStats(const bool print_trainstats) { (void)print_trainstats; }
  virtual void SetPrintResidualStats(const bool print_residualstats) {
    (void)print_residualstats;
  }
  virtual void SetPrintVarStats(const bool print_varstats) { (void)print_varstats; }

  // Host-side N(0, stdev) fill in memory order (recommender.h:61-67).  The
  // GPU models seed their device embeddings through frecsys_init_embeddings
  // with the identical generator; this stays for API compatibility.
  void init_matrix(MatrixXf* matrix, std::mt19937& gen, const float adjusted_stdev) {
    std::normal_distribution<float> d(0, adjusted_stdev);
    for (int64_t i = 0; i < matrix->size(); ++i) *(matrix->data() + i) = d(gen);
  }

  UserEvaluationResult EvaluateUser(const int num_items, const VectorXi& k_list,
                                    const VectorXf& all_scores, const SpVector& ground_truth,
                                    const SpVector& exclude) {
    VectorXf scores = all_scores;
    for (const auto& p : exclude) scores[p.first] = std::numeric_limits<float>::lowest();
    const int max_k = std::min<int>(k_list.maxCoeff(), (int)scores.size());
    std::vector<size_t> topk(scores.size());
    std::iota(topk.begin(), topk.end(), 0);
    auto greater = [&scores](size_t a, size_t b) { return scores[a] > scores[b]; };
    std::nth_element(topk.begin(), topk.begin() + max_k, topk.end(), greater);
    std::stable_sort(topk.begin(), topk.begin() + max_k, greater);
    (void)num_items;
    return RankMetrics(k_list, topk.data(), max_k, ground_truth);
  }

  // Recall@K and NDCG@K of a ranked list (recommender.h:152-182).
  template <typename Id>
  static UserEvaluationResult RankMetrics(const VectorXi& k_list, const Id* topk, int max_k,
                                          const SpVector& ground_truth) {
    std::set<int> gt;
    for (const auto& p : ground_truth) gt.insert(p.first);
    const int64_t nk = k_list.size();
    UserEvaluationResult r{VectorXf(nk), VectorXf(nk)};
    for (int64_t i = 0; i < nk; ++i) {
      const int k = std::min<int>(k_list[i], max_k);
      double hits = 0.0, dcg = 0.0, norm = 0.0;
      for (int j = 0; j < k; ++j)
        if (gt.count((int)topk[j])) {
          hits += 1.0;
          dcg += 1.0 / std::log2(j + 2.0);
        }
      const int m = std::min<int>(k_list[i], (int)gt.size());
      for (int j = 0; j < m; ++j) norm += 1.0 / std::log2(j + 2.0);
      r.recall[i] = (float)(hits / std::min<float>((float)k_list[i], (float)gt.size()));
      r.ndcg[i] = (float)(dcg / norm);
    }
    return r;
  }

  // Work-queue evaluation over eval_by_user (recommender.h:78-129).
  template <typename F>
  EvaluationResult EvaluateDatasetInternal(const int num_items, const VectorXi& k_list,
                                           const VectorXf& alpha_list,
                                           const std::unordered_map<int, int>& user_to_ind,
                                           const Dataset& data, const SpMatrix& eval_by_user,
                                           F score_user_and_history) {
    const int64_t nk = k_list.size();
    const int64_t nu = (int64_t)eval_by_user.size();
    MatrixXf recall = MatrixXf::Zero(nu, nk), ndcg = MatrixXf::Zero(nu, nk);
    std::vector<std::pair<int, const SpVector*>> work;
    work.reserve(eval_by_user.size());
    for (const auto& kv : eval_by_user) work.push_back({kv.first, &kv.second});
    const SpMatrix& hist = data.by_user();
    std::atomic<size_t> next{0};
    auto worker = [&] {
      for (;;) {
        const size_t w = next.fetch_add(1);
        if (w >= work.size()) return;
        const int u = work[w].first;
        const SpVector& h = hist.at(u);
        const VectorXf scores = score_user_and_history(u, h);
        const UserEvaluationResult m = EvaluateUser(num_items, k_list, scores, *work[w].second, h);
        const int row = user_to_ind.at(u);
        for (int64_t i = 0; i < nk; ++i) {
          recall(row, i) += m.recall[i];
          ndcg(row, i) += m.ndcg[i];
        }
      }
    };
    const int nt = (int)std::max(1u, std::thread::hardware_concurrency());
    std::vector<std::thread> th;
    for (int i = 0; i < nt; ++i) th.emplace_back(worker);
    for (auto& t : th) t.join();
    return EvaluationResult{k_list, alpha_list, recall, ndcg};
  }
};

}  // namespace frecsys
