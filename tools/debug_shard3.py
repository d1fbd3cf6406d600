import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import fuse_ref
import clasfv_amd.synthetic as S
from clasfv_amd import dist as D, fuse_utils as FU
from clasfv_amd.model import R2plus1D_18_MotionNet
m = R2plus1D_18_MotionNet(pretrained=False)
def nv(T, seed): return torch.from_numpy(fuse_ref.zeroone_normalizer(S.echo_video(T, seed=seed))).cuda()
vids = [nv(T, 300 + T) for T in (70, 96, 45)]
ref0 = FU.segment_a_video_with_fusion_device(vids[0], m, num_clips=3, step=1, fuse_method="majority")
for subset in ([0], [0, 1], [0, 2]):
    got = D.segment_videos_sharded([vids[i] for i in subset], m, num_clips=3, step=1, fuse_method="majority")
    print("subset", subset, "video0 diff", int((got[0] != ref0).sum()), flush=True)
got = D.segment_videos_sharded([vids[0]], m, num_clips=3, step=1, fuse_method="majority", batch_size=1)
print("bs1 video0 diff", int((got[0] != ref0).sum()))
got = D.segment_videos_sharded([vids[0]], m, num_clips=3, step=1, fuse_method="majority", clip_fn=lambda c: m(c)[0])
print("clip_fn video0 diff", int((got[0] != ref0).sum()))
