import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import fuse_ref
import clasfv_amd.synthetic as S
from clasfv_amd import dist as D, fuse_utils as FU
from clasfv_amd.model import R2plus1D_18_MotionNet
m = R2plus1D_18_MotionNet(pretrained=False)
def nv(T, seed): return torch.from_numpy(fuse_ref.zeroone_normalizer(S.echo_video(T, seed=seed))).cuda()
v0 = nv(70, 370)
rec = {}
orig_pl, orig_fv, orig_rm, orig_bc = FU.pass_labels, FU.fuse_votes, FU.run_model, FU.build_clips
def tag(name, fn):
    def w(*a, **k):
        out = fn(*a, **k)
        rec.setdefault(name, []).append(([x.clone() if torch.is_tensor(x) else x for x in a], out.clone()))
        return out
    return w
FU.pass_labels = tag("pl", orig_pl); FU.fuse_votes = tag("fv", orig_fv); FU.run_model = tag("rm", orig_rm); FU.build_clips = tag("bc", orig_bc)
ref0 = FU.segment_a_video_with_fusion_device(v0, m, num_clips=3, step=1, fuse_method="majority")
got = D.segment_videos_sharded([v0], m, num_clips=3, step=1, fuse_method="majority")
for name in ("bc", "rm", "pl", "fv"):
    (a1, o1), (a2, o2) = rec[name][0], rec[name][1]
    print(name, "out equal", bool(o1.shape == o2.shape and torch.equal(o1, o2)), [type(x).__name__ if torch.is_tensor(x) else x for x in a1][1:], [x if not torch.is_tensor(x) else tuple(x.shape) for x in a2][1:])
    for i, (x, y) in enumerate(zip(a1, a2)):
        if torch.is_tensor(x):
            print("   arg", i, tuple(x.shape), tuple(y.shape), bool(x.shape == y.shape and torch.equal(x, y)), x.dtype, y.dtype)
