"""MI355X-native CLAS-FV inference engine (import name ``clasfv_amd``).

Hot path of yc015/fully-automated-multi-heartbeat-echocardiography-video-segmentation-and-motion-tracking:
the R(2+1)D-18 encoder-decoder forward of ``R2plus1D_18_MotionNet`` over sliding 32-frame clips and
the per-clip softmax -> temporal re-interpolation -> argmax -> overlapping-clip label fusion of
``src/fuse_utils.py``, as hand-written HIP kernels for gfx950 behind a C ABI (include/clasfv.h,
libclasfv.so). Modules:

  model       R2plus1D_18_MotionNet drop-in (forward(x) -> (seg, motion))
  fuse_utils  divide_to_consecutive_clips / segment_a_video_with_fusion drop-ins
  warp        motion-field warp (generate_2dmotion_field + grid_sample semantics)
  echo        EF from masks (compute_ef_using_putative_clips, get2dPucks, EDESpairs)
  preprocess  zeroone_normalizer on the device
  dist        clip-wise sharding over ranks + all-gather of per-clip logits
"""
__version__ = "0.1.0"
