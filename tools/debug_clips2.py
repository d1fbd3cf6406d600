import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import fuse_ref
import clasfv_amd.synthetic as S
from clasfv_amd import fuse_utils as FU
vn = fuse_ref.zeroone_normalizer(S.echo_video(70, seed=370))
print(vn.shape, vn.dtype, vn.flags['C_CONTIGUOUS'], vn.strides)
a = FU.divide_to_consecutive_clips(vn, interpolate_last=True).cpu().numpy()
vt = torch.from_numpy(vn)
print(vt.shape, vt.stride(), vt.is_contiguous())
vc = vt.cuda()
print(vc.stride(), vc.is_contiguous())
b = FU.build_clips(vc, FU.clip_table(70, 1, 1)[0]).cpu().numpy()
exp = fuse_ref.divide_to_consecutive_clips(vn, interpolate_last=True)
print("numpy-path vs oracle", int((a != exp).sum()), " device-path vs oracle", int((b != exp).sum()), " a vs b", int((a != b).sum()))
print(float(np.abs(vc.cpu().numpy() - vn).max()))
