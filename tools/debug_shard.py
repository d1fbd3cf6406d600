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
for method in ("majority", "simple"):
    got = D.segment_videos_sharded(vids, m, num_clips=3, step=1, fuse_method=method)
    for i, v in enumerate(vids):
        ref = FU.segment_a_video_with_fusion_device(v, m, num_clips=3, step=1, fuse_method=method)
        ref2 = FU.segment_a_video_with_fusion_device(v, m, num_clips=3, step=1, fuse_method=method)
        d = (got[i] != ref)
        frames = torch.nonzero(d.flatten(1).any(1)).flatten().tolist()
        print(method, "video", i, "T", v.shape[1], "diff pixels", int(d.sum()), "frames", frames[:20], "ref-vs-ref2", int((ref != ref2).sum()), flush=True)
# logits comparison
plans, n_total = D.global_clip_plan([v.shape[1] for v in vids], 3, 1)
lg_all = D.run_clip_shard(n_total, 0, 1, lambda lo, hi: FU.run_model(m, torch.cat([FU.build_clips(vids[i], p["table"]) for i, p in enumerate(plans)])), None)
for i, p in enumerate(plans):
    clips = FU.build_clips(vids[i], p["table"])
    lg = FU.run_model(m, clips)
    print("video", i, "logit diff", int((lg != lg_all[p["offset"]:p["offset"] + p["n"]]).sum()), flush=True)
