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
plans, n_total = D.global_clip_plan([v.shape[1] for v in vids], 3, 1)
p = plans[0]
clips_all = torch.cat([FU.build_clips(vids[i], q["table"]) for i, q in enumerate(plans)])
lg_all = FU.run_model(m, clips_all)
lg_s = lg_all[p["offset"]:p["offset"] + p["n"]]
lg_v = FU.run_model(m, FU.build_clips(vids[0], p["table"]))
print("logits equal", bool(torch.equal(lg_s, lg_v)), lg_s.is_contiguous(), lg_s.data_ptr() == lg_all.data_ptr())
L1 = FU.pass_labels(lg_s, p["clip0"], p["T"], 1)
L2 = FU.pass_labels(lg_v, p["clip0"], p["T"], 1)
L3 = FU.pass_labels(lg_s.clone(), p["clip0"], p["T"], 1)
for k in range(p["K"]):
    tk = p["T"] - k
    print("pass", k, "diff s/v", int((L1[k, :tk] != L2[k, :tk]).sum()), "diff clone", int((L3[k, :tk] != L2[k, :tk]).sum()))
print("clip0", p["clip0"], "T", p["T"], "K", p["K"], "n", p["n"])
