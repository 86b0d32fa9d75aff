// Host-side launch API of the gfx950 kernels (raw pointers + stream; no torch headers,
// so every .hip compiles in seconds and the kernels are reusable from the C++ runtime).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct CsTensorEntry {
  float* p;
  float* g;
  float* m;
  int64_t n;
};

// data pipeline
hipError_t cs_augment(const uint8_t* data, const int64_t* idx, const int32_t* params, float* out, int B, int nhwc,
                      int cstride, const float* mean, const float* std_, hipStream_t stream);

// optimizer
hipError_t cs_sgd_flat(float* p, const float* g, float* m, int64_t n, float lr, float mom, float wd, float damp,
                       float scale, int first, hipStream_t stream);
hipError_t cs_sgd_multi(const CsTensorEntry* tab_dev, int ntens, const int64_t* chunk_start_dev, int nchunks,
                        float lr, float mom, float wd, float damp, float scale, int first, hipStream_t stream);

// classifier head
hipError_t cs_linear_xent(const float* feat, const float* W, const float* bias, const int64_t* labels, int B, int K,
                          int C, float gscale, float* loss_out, int* correct_out, float* logits_out, float* dW,
                          float* db, float* dfeat, int64_t* pred_out, hipStream_t stream);
hipError_t cs_softmax_xent(const float* logits, const int64_t* labels, int B, int C, float gscale, float* loss_out,
                           float* dlogits, int* correct_out, hipStream_t stream);
