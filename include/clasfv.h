/*
 * clasfv.h -- C ABI of the MI355X-native CLAS-FV engine (libclasfv.so, gfx950).
 *
 * Drop-in boundary for the reference hot path (yc015/fully-automated-multi-heartbeat-echocardiography-
 * video-segmentation-and-motion-tracking @ /root/reference):
 *   model forward      R2plus1D_18_MotionNet.forward(x) -> (seg, motion)
 *                        src/model/R2plus1D_18_MotionNet.py:26-71
 *   checkpoint load    model.load_state_dict(torch.load(path)["model"])    motion_segment.py:69-72
 *   clip plumbing      divide_to_consecutive_clips / segment_a_video_with_fusion
 *                        src/fuse_utils.py:16-100
 *   motion warp        generate_2dmotion_field + F.grid_sample(border, align_corners=False)
 *                        src/transform_utils.py:14-34, src/visualization_utils.py:128
 *   normaliser         zeroone_normalizer                                  src/echonet_dataset.py:38-50
 *
 * Conventions
 *   - Plain C types only. Tensors are dense row-major fp32 (labels: uint8) in the reference's
 *     layouts (N,C,T,H,W). Pointers marked _dev are device (HBM) pointers owned by the caller;
 *     the library owns weights and its workspace.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream). All launches are
 *     stream-ordered and asynchronous; no call synchronises the device except clasfv_finalize.
 *   - Every function returns CLASFV_OK (0) or a negative error code; clasfv_last_error() returns
 *     a thread-local message for the last failure. A handle is not re-entrant: calls on one handle
 *     must be serialised by the caller (one handle per device per process).
 */
#ifndef CLASFV_H
#define CLASFV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  CLASFV_OK = 0,
  CLASFV_EINVAL = -1,     /* bad argument / unknown parameter name */
  CLASFV_EBADSHAPE = -2,  /* shape not supported: T % 8, H % 16, W % 16 must be 0 */
  CLASFV_ENOTREADY = -3,  /* forward before clasfv_finalize / missing parameters */
  CLASFV_EHIP = -4,       /* HIP runtime error (message in clasfv_last_error) */
  CLASFV_ENOMEM = -5
};

/* ABI revision: bumped whenever an exported function changes its parameter list. Callers check
 * clasfv_version() == CLASFV_ABI_VERSION after loading the library (the ctypes binding does).
 *   1  round 1
 *   2  clasfv_zeroone_normalize takes a caller-owned workspace; clasfv_kernel_timing reports xgflop
 *   3  kernel variants (clasfv_set_kernel_variants), CLASFV_FUSE_FORCE_GENERIC */
#define CLASFV_ABI_VERSION 3

/* MAJORITY: ties -> 0; ITKVOTING: itk::LabelVotingImageFilter with its default undecided label
 * (max label + 1): ties -> 2. */
enum { CLASFV_FUSE_MAJORITY = 0, CLASFV_FUSE_SIMPLE = 1, CLASFV_FUSE_STAPLE = 2, CLASFV_FUSE_ITKVOTING = 3 };
/* OR-ed into a clasfv_fuse_votes method: run SIMPLE on its generic kernel instead of the packed
 * 16-vote one (A/B testing; results are identical). */
#define CLASFV_FUSE_FORCE_GENERIC 0x100
enum { CLASFV_DTYPE_FP32 = 0, CLASFV_DTYPE_BF16 = 1 };

/* Kernel-variant switches (A/B testing against the kernels each product kernel replaced; every
 * variant computes the same function -- NO_SPLIT_K the same sums in another fp32 summation order,
 * NO_WINO4 the same convolutions through F(2x2,3x3) instead of F(4x4,3x3) fp32 rounding).
 * Read once, at clasfv_create, from the environment variable named in the comment (set = on), or set
 * with clasfv_set_kernel_variants. Bits 131072, 1048576, 2097152, 8388608 and 33554432 are retired
 * (round-5 A/B forms that measured slower; they live only in tools/convbench now) and rejected. */
enum {
  CLASFV_VARIANT_NO_WINOGRAD = 1,      /* CLASFV_WINOGRAD=0: fp32 stride-1 convs on the direct implicit GEMM */
  CLASFV_VARIANT_NO_WINO_PATCH = 2,    /* CLASFV_NO_WINO_PATCH: conv_wino instead of conv_wino_q */
  CLASFV_VARIANT_WINOT_REFERENCE = 4,  /* CLASFV_WINOT_REFERENCE: conv_winot instead of conv_winot5 */
  CLASFV_VARIANT_NO_C8 = 8,            /* CLASFV_NO_C8: channels-last mid tensors everywhere */
  CLASFV_VARIANT_NO_STEM_BF16 = 16,    /* CLASFV_NO_STEM_BF16: bf16 engines run the fp32 stem */
  CLASFV_VARIANT_NO_PATCH_BF16 = 32,   /* CLASFV_NO_PATCH_BF16: bf16 stride-1 convs on conv_dma */
  CLASFV_VARIANT_NO_DECODER_BF16 = 64, /* CLASFV_NO_DECODER_BF16: bf16 engines run the fp32 decoder */
  CLASFV_VARIANT_WINOT_NO_TS1 = 128,   /* CLASFV_WINOT_TS1=0: T % 8 != 0 temporal convs on conv_winot */
  CLASFV_VARIANT_NO_SPLIT_K = 256,     /* CLASFV_NO_SPLIT_K: conv_winot5 grids smaller than the chip unsplit */
  CLASFV_VARIANT_NO_WINO4 = 512,       /* CLASFV_NO_WINO4: conv_wino_q (F(2x2,3x3)) instead of conv_wino4 (F(4x4,3x3)) */
  CLASFV_VARIANT_NO_DECODER_X3 = 1024, /* CLASFV_NO_DECODER_X3: fp32 engines run comb_2 on fp32 MFMAs, not split bf16 */
  CLASFV_VARIANT_NO_DMA_X3 = 2048,     /* CLASFV_NO_DMA_X3: fp32 strided / 1x1x1 convs on conv_dma (fp32 MFMA), not conv_dma_x3 */
  CLASFV_VARIANT_NO_STEM_X3 = 4096,    /* CLASFV_NO_STEM_X3: fp32 engines' stem on conv_stem_f32 (fp32 MFMA), not conv_stem_x3 */
  CLASFV_VARIANT_NO_WINO4W = 8192,     /* CLASFV_NO_WINO4W: conv_wino4 (48-channel blocks) instead of conv_wino4w (wide blocks) */
  CLASFV_VARIANT_NO_PATCH32 = 16384,   /* CLASFV_NO_PATCH32: bf16 1x3x3 convs on conv_patch_bf16 (16x16x32 tiles) instead of conv_patch32_bf16 (32x32x16) */
  CLASFV_VARIANT_NO_PROJ_X3 = 32768,   /* CLASFV_NO_PROJ_X3: the decoder's 128-deep tap projections on conv_dma_x3 instead of the persistent conv_proj_x3 */
  CLASFV_VARIANT_NO_WINO4R = 65536,    /* CLASFV_NO_WINO4R: wide-block 1x3x3 convs on conv_wino4w (4 quadrant waves, one per SIMD) instead of conv_wino4r (12 row waves, three per SIMD) */
  CLASFV_VARIANT_NO_DMA_BUF = 262144,  /* CLASFV_NO_DMA_BUF: conv_dma_x3's LDS-DMAs from 64-bit pointers instead of 32-bit buffer offsets */
  CLASFV_VARIANT_W4R_CACHED_STORES = 524288, /* CLASFV_W4R_CACHED_STORES: conv_wino4r's output stores cached instead of non-temporal */
  CLASFV_VARIANT_PATCH32_CACHED_STORES = 4194304, /* CLASFV_PATCH32_CACHED_STORES: conv_patch32_bf16's output stores cached (the product's are non-temporal) */
  CLASFV_VARIANT_NO_DMA_W = 16777216,       /* CLASFV_NO_DMA_W: the bf16 engines' direct convs on conv_dma (64-B LDS rows) instead of conv_dma_w (128-B rows) */
  CLASFV_VARIANT_NO_TWALK = 67108864        /* CLASFV_NO_TWALK: the bf16 engines' 64-channel temporal convs (layer1, stem) on conv_patch_bf16 instead of the frame-walking conv_twalk_bf16 (round 6) */
};

typedef struct clasfv_engine* clasfv_t;

const char* clasfv_last_error(void);
/* CLASFV_ABI_VERSION of the loaded library. */
int clasfv_version(void);
/* Content hash of the sources the library was compiled from ("clasfv-source-hash:<16 hex>",
 * computed by the build over csrc/ and this header): a binding can refuse a library older than its
 * sources without trusting file times. Does not change the ABI revision (a new export only). */
const char* clasfv_source_hash(void);

/* ---- model: replaces R2plus1D_18_MotionNet.__init__/load_state_dict/forward ------------------ */
int clasfv_create(int device, clasfv_t* out);
int clasfv_destroy(clasfv_t h);
/* Number / name / shape of the 242 state-dict entries the engine accepts (reference key names,
 * e.g. "r2plus1d_model.stem.0.weight"); shape is written to dims[0..*ndim). */
int clasfv_param_count(clasfv_t h);
int clasfv_param_info(clasfv_t h, int i, const char** name, int* ndim, int64_t dims[5]);
/* Copy one state-dict entry from host memory. A "module." prefix (nn.DataParallel checkpoints,
 * motion_segment.py:69) is accepted. num_batches_tracked entries are accepted and ignored. */
int clasfv_load_param(clasfv_t h, const char* name, const float* host_data, int64_t numel);
/* Fold eval-mode BatchNorm into the convolutions, pad channels for the kernels, upload to HBM. */
int clasfv_finalize(clasfv_t h);
/* seg_dev (N,2,T,H,W) logits and motion_dev (N,4,T,H,W) tanh outputs from x_dev (N,3,T,H,W).
   Stream-ordered on `stream` (a hipStream_t; NULL = the default stream), no host synchronisation.
   The handle keeps one workspace per launch stream (up to 4; a fifth stream takes over the least
   recently used one after a device synchronisation), so forwards issued on different streams may run
   concurrently; calls on one handle must come from one host thread at a time. */
int clasfv_forward(clasfv_t h, const float* x_dev, int N, int T, int H, int W, float* seg_dev,
                   float* motion_dev, void* stream);
/* Bytes of library workspace currently held (the per-stream activation arenas; each grows to the
   largest N*T*H*W seen on its stream). */
int64_t clasfv_workspace_bytes(clasfv_t h);
/* Compute dtype of the encoder: CLASFV_DTYPE_FP32 (default; exact-fp32 MFMA, the reference's
 * precision) or CLASFV_DTYPE_BF16 (bf16 activations/weights, fp32 accumulation; BASELINE config[4],
 * Dice tolerance 1e-2). The decoder head runs in fp32 either way. A change takes effect at the next
 * clasfv_finalize. */
int clasfv_set_compute_dtype(clasfv_t h, int dtype);
int clasfv_get_compute_dtype(clasfv_t h);
/* Kernel-variant switches (CLASFV_VARIANT_* bits). A change of CLASFV_VARIANT_NO_WINOGRAD needs the
 * next clasfv_finalize (the Winograd weight images are built there); the others apply to the next
 * clasfv_forward. */
int clasfv_set_kernel_variants(clasfv_t h, int flags);
int clasfv_get_kernel_variants(clasfv_t h);

/* ---- instrumentation (bench.py's live roofline; not on the reference's interface) ------------ */
/* enable != 0: every later clasfv_forward records one HIP event on its stream before its first
 * launch and one after each launch, so each kernel's device time is the gap between two events.
 * Enabling or disabling drops what was recorded. */
int clasfv_set_kernel_timing(clasfv_t h, int enable);
/* Waits for the recorded events, aggregates the launches recorded since the last call per kernel
 * and clears them. Entry i: names[i] (static string, e.g. "conv_wino"), launches[i], ms[i] (summed
 * device time), gflop[i] (summed algorithmic GFLOP, 2 per MAC over unpadded channels: the direct
 * convolution the launch replaces), xgflop[i] (summed GFLOP the launch issues to the matrix cores:
 * Winograd-domain products, padded channels and partial tiles included -- the roofline numerator).
 * Returns the number of entries (<= cap) or a negative error code. */
int clasfv_kernel_timing(clasfv_t h, int cap, const char** names, int* launches, double* ms,
                         double* gflop, double* xgflop);

/* ---- clip plumbing: replaces src/fuse_utils.py:16-100 ----------------------------------------- */
/* Build n clips (n,3,32,H,W) from the normalised video (3,T,H,W). Clip i is frames
 * [table[2i+1], table[2i+1]+32) of the temporally shifted video video[:, table[2i]:], resampled
 * to 32*round(T_k/32) frames (align_corners=False, as F.interpolate) when interpolate != 0 and
 * T_k % 32 != 0. table_dev is a device int32 array of 2n entries. */
int clasfv_build_clips(const float* video_dev, int T, int H, int W, const int32_t* table_dev, int n,
                       int interpolate, float* clips_dev, void* stream);
/* For each shifted pass k < K: softmax over the 2 classes of the pass's clips' logits
 * (logits_dev + pass_clip0[k] clips, each (2,32,H,W)), resample to T_k = T - k*step frames
 * (align_corners=False) when T_k % 32 != 0 and interpolate != 0, argmax -> labels_dev[k][0..T_k)
 * (labels_dev is (K,T,H,W) uint8). pass_clip0 is a host array of K ints. */
int clasfv_pass_labels(const float* logits_dev, int K, const int32_t* pass_clip0, int T, int step, int H,
                       int W, int interpolate, uint8_t* labels_dev, void* stream);
/* Same labels from logit margins d = l1 - l0 ((n,32,H,W) per clip, clasfv_logit_margin) instead of
 * the two logit planes: bit-identical, because the 2-class softmax depends on the logits only
 * through fl(l1 - l0). Used for the multi-GPU exchange (half the bytes on xGMI). */
int clasfv_pass_labels_margin(const float* margin_dev, int K, const int32_t* pass_clip0, int T, int step,
                              int H, int W, int interpolate, uint8_t* labels_dev, void* stream);
/* margin_dev (n,32,H,W) = logits_dev[:,1] - logits_dev[:,0] for n clips of (2,32,H,W) logits. */
int clasfv_logit_margin(const float* logits_dev, int n, int H, int W, float* margin_dev, void* stream);
/* Per-frame label fusion over the K <= 64 shifted passes (fuse_utils.py:82-100). Output (T',H,W)
 * uint8 with T' = T - (step - 1). method: CLASFV_FUSE_MAJORITY, CLASFV_FUSE_SIMPLE,
 * CLASFV_FUSE_STAPLE or CLASFV_FUSE_ITKVOTING (LabelFusion's methods, fuse_utils.py:95; SIMPLE,
 * STAPLE and ITK voting are restated from their published definitions: LabelFusion itself is absent,
 * so their parity is unpinned). */
int clasfv_fuse_votes(const uint8_t* labels_dev, int K, int T, int step, int H, int W, int method,
                      uint8_t* fused_dev, void* stream);

/* ---- motion warp (src/transform_utils.py:14-34 + grid_sample) ------------------------------------ */
/* out (N,C,H,W) = bilinear sample of img at (linspace_W[j] + motion[n,0,i,j],
 * linspace_H[i] + motion[n,1,i,j]), border padding, align_corners=False. motion is (N,2,H,W) with
 * arbitrary element strides for n and the channel (so a slice motion[:, 0:2, t] of (N,4,T,H,W) can
 * be passed directly): element (n,c,i,j) at motion_dev[n*m_sn + c*m_sc + i*W + j]. */
int clasfv_warp(const float* img_dev, int N, int C, int H, int W, const float* motion_dev, int64_t m_sn,
                int64_t m_sc, float* out_dev, void* stream);

/* Gradients of clasfv_warp (training losses, src/clasfv_losses.py:29-136, backpropagate through it):
 * grad_img_dev (N,C,H,W) += d loss / d img (atomically accumulated: zero it first; may be NULL),
 * grad_motion_dev (N,2,H,W) dense = d loss / d motion (may be NULL), from grad_out_dev (N,C,H,W).
 * grad_motion is bit-exact vs PyTorch's CPU grid_sample backward; grad_img matches it to float
 * rounding (different summation order). motion strides as in clasfv_warp. */
int clasfv_warp_backward(const float* grad_out_dev, const float* img_dev, int N, int C, int H, int W,
                         const float* motion_dev, int64_t m_sn, int64_t m_sc, float* grad_img_dev,
                         float* grad_motion_dev, void* stream);

/* ---- preprocessing (motion_segment.py:96-106, src/echonet_dataset.py:38-50) --------------------- */
/* frames_dev (T,Hs,Ws,3) uint8 RGB -> out_dev (3,T,H,W) float32, resized as
 * F.interpolate(size=(T,H,W), mode="trilinear", align_corners=True) on the (1,3,T,Hs,Ws) float
 * video (bit-exact vs PyTorch's CPU kernel). Not normalised: follow with clasfv_zeroone_normalize. */
int clasfv_preprocess_video(const uint8_t* frames_dev, int T, int Hs, int Ws, int H, int W, float* out_dev,
                            void* stream);
/* In place: per channel c of video (3, n_per_channel) subtract the channel min, divide by the max.
 * workspace_dev: caller-owned device scratch of clasfv_zeroone_workspace_bytes() bytes, used in
 * stream order (concurrent calls on different streams need different workspaces). */
int64_t clasfv_zeroone_workspace_bytes(void);
int clasfv_zeroone_normalize(float* video_dev, int64_t n_per_channel, float* workspace_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CLASFV_H */
