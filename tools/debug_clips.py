import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import fuse_ref
import clasfv_amd.synthetic as S
from clasfv_amd import fuse_utils as FU
v = torch.from_numpy(fuse_ref.zeroone_normalizer(S.echo_video(70, seed=370))).cuda()
table, clip0 = FU.clip_table(70, 3, 1)
ref = fuse_ref.divide_to_consecutive_clips  # per pass
outs = [FU.build_clips(v, table) for _ in range(4)]
torch.cuda.synchronize()
for i, o in enumerate(outs):
    print("call", i, "diff vs call0", int((o != outs[0]).sum()))
vn = v.cpu().numpy()
exp = np.concatenate([fuse_ref.divide_to_consecutive_clips(vn[:, s:], interpolate_last=True) for s in range(3)])
for i, o in enumerate(outs):
    d = (o.cpu().numpy() != exp)
    print("call", i, "diff vs oracle", int(d.sum()), "per clip", d.reshape(6, -1).sum(1).tolist())
