// Classification bookkeeping on device: the per-batch work of AVMNIST.train_step / validation_step
// after the loss (MML_Suite/models/avmnist.py:305-309,345-350: softmax → argmax → .cpu() →
// MetricRecorder.update_group_all, experiment_utils/metric_recorder.py:96-145) and of the epoch loops'
// loss lists (train_multimodal.py:478-491,525-541), without a host round trip per batch:
//   pred[r] = first argmax of softmax(logits[r]);  confusion[group[r]][label[r]][pred[r]] += 1
//   loss_log[counters[0]++] = *loss;  counters[1] += n
// The monomodal pre-training step predicts argmax(logits) instead (train_monomodal.py:236,394):
// tspm_classify_update_ex(..., TSPM_ARGMAX_LOGITS, ...).
// Every metric the reference's YAML names (accuracy, balanced accuracy, precision / recall / F1 with
// macro / micro / weighted averaging, the confusion matrix) is a function of the per-group confusion
// counts, evaluated at epoch end on the host (metrics.py).  Integer atomics: order-independent.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void k_classify_update(int N, int K, const float* __restrict__ logits,
                                                         const long long* __restrict__ labels,
                                                         const int* __restrict__ groups, int G,
                                                         unsigned long long* __restrict__ conf,
                                                         long long* __restrict__ pred_out,
                                                         const float* __restrict__ loss, float* __restrict__ loss_log,
                                                         long long* __restrict__ counters, long long cap,
                                                         int on_logits) {
  for (int n = blockIdx.x * 256 + threadIdx.x; n < N; n += gridDim.x * 256) {
    const float* z = logits + (long long)n * K;
    int am = 0;
    if (on_logits) {
      // torch.argmax(logits, 1): the first maximal logit
      float best = z[0];
      for (int k = 1; k < K; ++k)
        if (z[k] > best) { best = z[k]; am = k; }
    } else {
      float mx = z[0];
      for (int k = 1; k < K; ++k) mx = fmaxf(mx, z[k]);
      float se = 0.f;
      for (int k = 0; k < K; ++k) se += expf(z[k] - mx);
      // argmax over the softmax values themselves (two logits 1 ulp apart can round to one
      // probability; the reference takes the first of those)
      float best = expf(z[0] - mx) / se;
      for (int k = 1; k < K; ++k) {
        const float p = expf(z[k] - mx) / se;
        if (p > best) { best = p; am = k; }
      }
    }
    if (pred_out) pred_out[n] = am;
    const long long lab = labels[n];
    const int g = groups ? groups[n] : 0;
    if (conf && lab >= 0 && lab < K && g >= 0 && g < G)
      atomicAdd(conf + ((long long)g * K + lab) * K + am, 1ULL);
  }
  if (counters && blockIdx.x == 0 && threadIdx.x == 0) {
    const long long b = counters[0];
    if (loss_log && loss && b < cap) loss_log[b] = *loss;
    counters[0] = b + 1;
    __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(counters + 1), (unsigned long long)N,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

extern "C" int tspm_classify_update_ex(int32_t n, int32_t classes, const float* logits, const int64_t* labels,
                                       const int32_t* groups, int32_t n_groups, int64_t* confusion, int64_t* pred_out,
                                       const float* loss, float* loss_log, int64_t* counters, int64_t log_capacity,
                                       int32_t argmax_of, tspm_stream_t stream) {
  if (n < 0 || classes <= 0 || n_groups <= 0 || log_capacity < 0) return TSPM_ERR_INVALID;
  if (argmax_of != TSPM_ARGMAX_SOFTMAX && argmax_of != TSPM_ARGMAX_LOGITS) return TSPM_ERR_INVALID;
  if (n > 0 && (!logits || !labels)) return TSPM_ERR_INVALID;
  if (loss_log && (!loss || !counters)) return TSPM_ERR_INVALID;
  if (n == 0 && !counters) return TSPM_OK;
  const int blocks = n > 0 ? (int)std::min<long long>(cdiv64(n, 256), 64) : 1;
  hipLaunchKernelGGL(k_classify_update, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), n, classes,
                     logits, reinterpret_cast<const long long*>(labels), groups, n_groups,
                     reinterpret_cast<unsigned long long*>(confusion), reinterpret_cast<long long*>(pred_out), loss,
                     loss_log, reinterpret_cast<long long*>(counters), (long long)log_capacity,
                     argmax_of == TSPM_ARGMAX_LOGITS ? 1 : 0);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_classify_update(int32_t n, int32_t classes, const float* logits, const int64_t* labels,
                                    const int32_t* groups, int32_t n_groups, int64_t* confusion, int64_t* pred_out,
                                    const float* loss, float* loss_log, int64_t* counters, int64_t log_capacity,
                                    tspm_stream_t stream) {
  return tspm_classify_update_ex(n, classes, logits, labels, groups, n_groups, confusion, pred_out, loss, loss_log,
                                 counters, log_capacity, TSPM_ARGMAX_SOFTMAX, stream);
}
