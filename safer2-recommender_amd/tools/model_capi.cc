// model_capi.cc -- libfrecsys_model.so, the C-ABI of include/frecsys_model.h
// over the C++ model classes (include/frecsys/*.h).  A thin owner of one
// Dataset + one Recommender built by the run_model factory
// (frecsys/factory.h); every compute call lands in libfrecsys_hip.so.
#include <array>
#include <cmath>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "frecsys/factory.h"
#include "frecsys_model.h"

struct frecsys_model {
  std::string name;
  std::unique_ptr<frecsys::Dataset> train;
  std::unique_ptr<frecsys::Recommender> rec;
};

namespace {
std::string g_model_error;
int model_fail(int code, const std::string& msg) {
  g_model_error = msg;
  return code;
}
}  // namespace

extern "C" {

void frecsys_model_config_default(frecsys_model_config* c) {
  if (!c) return;
  std::memset(c, 0, sizeof(*c));
  const frecsys::ModelParams p;  // run_model.cc:129-230 defaults
  c->dim = p.dim;
  c->l2_reg = p.l2_reg;
  c->l2_reg_exp = p.l2_reg_exp;
  c->uobs_weight = p.uobs_weight;
  c->stdev = p.stdev;
  c->alpha = p.alpha;
  c->bandwidth = p.bandwidth;
  c->stepsize = p.stepsize;
  c->sampling_ratio = p.sampling_ratio;
  c->block_size = p.block_size;
  c->xi_iterations = p.xi_iterations;
  c->pd_iterations = p.pd_iterations;
  c->use_epanechnikov = p.use_epanechnikov;
  c->use_snr = p.use_snr;
  c->print_train_stats = p.print_train_stats;
  c->print_residual_stats = p.print_residual_stats;
  c->print_var_stats = p.print_var_stats;
  c->seed = -1;
  c->device = -1;
  c->parity_quirks = 1;
  c->world = 0;
  c->rank = -1;
  c->comm_id = nullptr;
}

int frecsys_model_create(const frecsys_model_config* c, const int32_t* users, const int32_t* items,
                         int64_t n_tuples, frecsys_model** out) {
  if (!c || !out || n_tuples <= 0 || !users || !items || !c->model_name)
    return model_fail(FRECSYS_ERR_INVALID, "frecsys_model_create: bad arguments");
  *out = nullptr;
  const std::string name = c->model_name;
  if (!frecsys::IsKnownModel(name))
    return model_fail(FRECSYS_ERR_INVALID, "unknown model " + name);
  if (frecsys_padded_dim(c->dim) == 0)
    return model_fail(FRECSYS_ERR_UNSUPPORTED, "dim " + std::to_string(c->dim) + " not built");
  for (int64_t k = 0; k < n_tuples; ++k)
    if (users[k] < 0 || items[k] < 0)
      return model_fail(FRECSYS_ERR_INVALID, "negative id in tuple " + std::to_string(k));
  int32_t ndev = 0;  // the C++ layer aborts on a missing device; report it instead
  if (frecsys_device_count(&ndev) != FRECSYS_OK || ndev == 0)
    return model_fail(FRECSYS_ERR_NO_DEVICE, "no HIP device visible");
  frecsys::ModelParams p;
  p.dim = c->dim;
  p.l2_reg = c->l2_reg;
  p.l2_reg_exp = c->l2_reg_exp;
  p.uobs_weight = c->uobs_weight;
  p.stdev = c->stdev;
  p.alpha = c->alpha;
  p.bandwidth = c->bandwidth;
  p.stepsize = c->stepsize;
  p.sampling_ratio = c->sampling_ratio;
  p.block_size = c->block_size;
  p.xi_iterations = c->xi_iterations;
  p.pd_iterations = c->pd_iterations;
  p.use_epanechnikov = c->use_epanechnikov != 0;
  p.use_snr = c->use_snr != 0;
  p.print_train_stats = c->print_train_stats != 0;
  p.print_residual_stats = c->print_residual_stats != 0;
  p.print_var_stats = c->print_var_stats != 0;
  frecsys::DeviceOptions o;
  o.seed = c->seed;
  o.device = c->device;
  o.parity_quirks = c->parity_quirks != 0;
  o.world = c->world;
  o.rank = c->rank;
  if (c->comm_id) {
    o.has_comm_id = true;
    std::memcpy(o.comm_id.data(), c->comm_id, 128);
  }
  auto m = std::make_unique<frecsys_model>();
  m->name = name;
  m->train = std::make_unique<frecsys::Dataset>(std::vector<int32_t>(users, users + n_tuples),
                                                std::vector<int32_t>(items, items + n_tuples));
  m->rec.reset(frecsys::MakeRecommender(name, m->train->max_user() + 1,
                                        m->train->max_item() + 1, p, o));
  *out = m.release();
  return FRECSYS_OK;
}

int frecsys_model_initialize(frecsys_model* m) {
  if (!m) return model_fail(FRECSYS_ERR_INVALID, "null model");
  frecsys::InitializeRecommender(m->name, m->rec.get(), *m->train);
  return FRECSYS_OK;
}

int frecsys_model_train(frecsys_model* m, int32_t epochs) {
  if (!m || epochs < 0) return model_fail(FRECSYS_ERR_INVALID, "frecsys_model_train: bad arguments");
  for (int32_t e = 0; e < epochs; ++e) m->rec->Train(*m->train);
  return FRECSYS_OK;
}

frecsys_ctx* frecsys_model_context(frecsys_model* m) {
  return m ? frecsys::AsDeviceModel(m->rec.get())->device().raw() : nullptr;
}

float frecsys_model_mean_weight(const frecsys_model* m) {
  if (!m) return NAN;
  frecsys::Recommender* r = m->rec.get();
  if (m->name == "safer2" || m->name == "safer2pp")
    return static_cast<frecsys::SAFER2Recommender*>(r)->GetMeanWeight();
  if (m->name == "erm_mf") return static_cast<frecsys::ERMMFRecommender*>(r)->GetMeanWeight();
  if (m->name == "cvar_mf") return static_cast<frecsys::CVaRMFRecommender*>(r)->GetMeanWeight();
  return NAN;
}

int frecsys_model_dual_state(const frecsys_model* m, float* weights, float* losses,
                             float* item_reg, float* xi) {
  if (!m) return model_fail(FRECSYS_ERR_INVALID, "null model");
  const frecsys::detail::DeviceModel* dm = frecsys::AsDeviceModel(m->rec.get());
  const frecsys::VectorXf& w = dm->dual_weights();
  if ((weights || item_reg) && w.size() == 0)
    return model_fail(FRECSYS_ERR_INVALID, m->name + " has no dual weights");
  if (weights) std::memcpy(weights, w.data(), sizeof(float) * (size_t)w.size());
  if (losses) {
    const frecsys::VectorXf& l = dm->user_loss();
    std::memcpy(losses, l.data(), sizeof(float) * (size_t)l.size());
  }
  if (item_reg) {
    const frecsys::VectorXf& r = dm->item_regularization();
    std::memcpy(item_reg, r.data(), sizeof(float) * (size_t)r.size());
  }
  if (xi) {
    *xi = NAN;
    if (m->name == "safer2" || m->name == "safer2pp")
      *xi = static_cast<const frecsys::SAFER2Recommender*>(m->rec.get())->xi();
  }
  return FRECSYS_OK;
}

void frecsys_model_destroy(frecsys_model* m) { delete m; }

const char* frecsys_model_last_error(void) { return g_model_error.c_str(); }

}  // extern "C"
