"""How many TESA candidates need a SAD on the bench workload: for 400 random MBs of the
synthetic 1080p pair with bench.tesa_params predictors, count the window candidates whose
ads4 value is below the predictor-bound threshold (bsad0 - ycost)*17>>4 (me.c:667-676).
CPU only (numpy); prints the per-MB mean / median / max."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from __graft_entry__ import load_package
x = load_package()
from x264hip import synth
import bench
W,H=1920,1088
planes, stride, origin = synth.make_sequence(2, W, H, 8)
ref = planes[0].astype(np.int64).reshape(-1, stride) if planes[0].ndim==1 else planes[0].astype(np.int64)
fenc = planes[1].astype(np.int64).reshape(ref.shape)
oy, ox = divmod(origin, stride)
mbw, mbh = W//16, H//16
par, init, cm, span = bench.tesa_params(mbw, mbh, 1, 16)
cm = cm.astype(np.int64)
# 8x8 box sums of ref at every position
c = np.zeros((ref.shape[0]+1, ref.shape[1]+1), np.int64); c[1:,1:] = ref.cumsum(0).cumsum(1)
def s8(y, x): return c[y+8, x+8] - c[y, x+8] - c[y+8, x] + c[y, x]
tot = need_tot = 0; needs=[]
rng = np.random.default_rng(0)
for mb in rng.choice(mbw*mbh, 400, replace=False):
    mbx, mby = mb % mbw, mb // mbw
    p = par[mb]
    bmx, bmy = int(p[0]), int(p[1])
    fy, fx = oy + 16*mby, ox + 16*mbx
    blk = fenc[fy:fy+16, fx:fx+16]
    dc = [blk[:8,:8].sum(), blk[:8,8:].sum(), blk[8:,:8].sum(), blk[8:,8:].sum()]
    min_x = max(bmx-16, int(p[4])); min_y = max(bmy-16, int(p[5]))
    max_x = min(bmx+16, int(p[6])); max_y = min(bmy+16, int(p[7]))
    width = (max_x - min_x + 3) & ~3
    cx = lambda mx: cm[span + 4*mx - int(p[2])]; cy = lambda my: cm[span + 4*my - int(p[3])]
    sad0 = np.abs(blk - ref[fy+bmy:fy+bmy+16, fx+bmx:fx+bmx+16]).sum()
    bsad0 = sad0 + cx(bmx) + cy(bmy)
    n = 0
    for my in range(min_y, max_y+1):
        yc = cy(my)
        if bsad0 <= yc: continue
        ub = (bsad0 - yc)*17 >> 4
        for mx in range(min_x, min_x+width):
            y, xx = fy+my, fx+mx
            ads = abs(dc[0]-s8(y,xx)) + abs(dc[1]-s8(y,xx+8)) + abs(dc[2]-s8(y+8,xx)) + abs(dc[3]-s8(y+8,xx+8)) + cx(mx)
            n += ads < ub
            tot += 1
    needs.append(n)
needs = np.array(needs)
print("candidates per MB", tot/len(needs), "need mean", needs.mean(), "median", np.median(needs), "max", needs.max(), "p90", np.percentile(needs,90))
