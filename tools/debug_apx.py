"""Debug helper: GPU double-approximate path vs the oracle on a small case; prints mismatches."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iron_weight_only_quant_amd import kernels as K
from oracle import approx_codec as A, fp_codec as C
from oracle.synth import synth

x = synth(403, (8, 64), "float16")
exp, s = A.quantlinear_approx(x, 4, 3, 32, 0, 12, 15, 1, True)
r = K.quantize_fp_approx(torch.from_numpy(x).cuda(), 4, 3, 32, 0, 12, 15, 1, True)
got = r.out.cpu().numpy()
print("scales equal", np.array_equal(r.scales.cpu().numpy(), s.reshape(-1)))
bad = np.argwhere(got.view(np.uint16) != exp.view(np.uint16))
print("bad", len(bad), "of", got.size)
sv = s.reshape(-1).astype(np.float32)
t = np.clip(C.R(x.reshape(-1, 32).astype(np.float64) / sv[:, None]), -480, 480)
codes = C.float_to_fp(t.astype(np.float16), 4, 3, 7)
for (i, j) in bad[:12]:
    g = (i * 64 + j) // 32
    print(i, j, "got", got[i, j], "exp", exp[i, j], "code", codes.reshape(8, 64)[i, j], "scale", sv[g])
