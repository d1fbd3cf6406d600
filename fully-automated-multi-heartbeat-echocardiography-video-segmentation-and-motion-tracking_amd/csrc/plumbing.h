// Launchers of the memory-bound pipeline kernels (plumbing.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CLASFV_MAX_PASSES 64

hipError_t launch_build_clips(const float* video, int T, int HW, const int32_t* table, int n, int interp, float* clips,
                              hipStream_t s);
hipError_t launch_pass_labels(const float* logits, int K, const int32_t* clip0, int T, int step, int HW, int interp,
                              int margin, uint8_t* labels, hipStream_t s);
hipError_t launch_logit_margin(const float* logits, int n, int HW, float* margin, hipStream_t s);
hipError_t launch_fuse_votes(const uint8_t* labels, int K, int T, int step, int HW, int method, uint8_t* fused,
                             hipStream_t s);
hipError_t launch_warp(const float* img, int N, int C, int H, int W, const float* motion, int64_t m_sn, int64_t m_sc,
                       float* out, hipStream_t s);
hipError_t launch_zeroone_normalize(float* v, int64_t n, float* part, hipStream_t s);
int zeroone_partials_floats();
hipError_t launch_preprocess_video(const uint8_t* frames, int T, int Hs, int Ws, int H, int W, float* out,
                                   hipStream_t s);
hipError_t launch_warp_backward(const float* gout, const float* img, int N, int C, int H, int W, const float* motion,
                                int64_t m_sn, int64_t m_sc, float* gimg, float* gmot, hipStream_t s);
