"""k_pis_net vs the layer-wise chain on one small HJB call: which row regions differ (A_0..A_3, GX).
usage: python tools/debug_pisnet.py [n M]"""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import deeppicarditeration_amd as dpi  # noqa: E402
from deeppicarditeration_amd import _lib as L  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
M = int(sys.argv[2]) if len(sys.argv) > 2 else 128
eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0, alpha_scale=4.0)
torch.manual_seed(0)
net = dpi.PISGradNet(hidden_shapes=[512] * 4, dim=100, g0=eq.g, T=1.0)
gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                              n_estimate_integral=M, n_euler_steps=8, seed=5)
tx, _ = gen.sample_t_and_x(n, point_base=0)
# x3 rows layout (pis_rows_layout, split): stride 4160 floats
REG = {"IN": (192, 192), "A0": (512, 512), "A1": (1024, 512), "A2": (1536, 512), "A3": (2048, 512), "GX": (3712, 128),
       "SS": (3840, 128), "ST": (3968, 128), "SC": (4096, 8)}
STRIDE = 4160
R = n * M + n
hb_off = 256 * ((n * 4 + 255) // 256) * 2 + 0
out = {}
for fused in ("0", "1", "1"):
    os.environ["DPI_PIS_FUSED"] = fused
    ws = gen.point_baseline(tx)
    mom = gen.label_moments(tx, 0, M, 0, M, L.DPI_BOTH, ws)
    torch.cuda.synchronize()
    f = ws.view(torch.float32) if ws.dtype != torch.float32 else ws
    out.setdefault(fused, []).append((mom.clone(), f.clone()))
# rows offset: gx, fb, bx (H = 0 for PISGradNet), hb (n * 128 floats)
al = lambda x: (x + 255) & ~255  # noqa: E731
rows_off = (al(n * 4) + al(n * 4) + al(0) + al(n * 128 * 4)) // 4
a, b, b2 = out["0"][0][1], out["1"][0][1], out["1"][1][1]
print("moments equal layer/fused:", torch.equal(out["0"][0][0], out["1"][0][0]), "fused/fused:",
      torch.equal(out["1"][0][0], out["1"][1][0]))
rows_a = a[rows_off:rows_off + R * STRIDE].view(R, STRIDE)
rows_b = b[rows_off:rows_off + R * STRIDE].view(R, STRIDE)
rows_b2 = b2[rows_off:rows_off + R * STRIDE].view(R, STRIDE)
def split_vals(rows, o, w):
    """split region words -> fp32 values: chunk u of 32 words = 4 granule pairs of (4 hi words, 4 lo words)"""
    v = rows[:, o:o + w].contiguous().view(torch.int32).view(R, w // 32, 4, 2, 4)
    h = v[:, :, :, 0, :].contiguous().view(torch.float16).float()
    lo = v[:, :, :, 1, :].contiguous().view(torch.float16).float()
    return h + lo


for k in ("A0", "A1", "A3", "GX"):
    o, w = REG[k]
    va, vb = split_vals(rows_a, o, w), split_vals(rows_b, o, w)
    d = (va - vb).abs()
    print(f"{k}: max |diff| {float(d.max()):.3e}  max |val| {float(va.abs().max()):.3e}  rel {float(d.max() / va.abs().max()):.3e}"
          f"  frac differing {float((d > 0).float().mean()):.3f}")
va, vb = split_vals(rows_a, 512, 512), split_vals(rows_b, 512, 512)  # A0 (R, 16 chunks, 4 pairs, 8)
d = (va != vb)
print("A0 differing fraction by chunk U:", [round(float(x), 2) for x in d.float().mean((0, 2, 3))])
print("A0 by granule pair q:", [round(float(x), 2) for x in d.float().mean((0, 1, 3))])
print("A0 by element j:", [round(float(x), 2) for x in d.float().mean((0, 1, 2))])
rm = torch.arange(R, device=d.device)
print("A0 by row % 64 // 16:", [round(float(d[(rm % 64) // 16 == k].float().mean()), 2) for k in range(4)])
print("A0 by row % 16:", [round(float(d[(rm % 16) == k].float().mean()), 2) for k in range(16)])
print("A0 row 0 chunk 0 layer:", [round(float(x), 4) for x in va[0, 0].flatten()[:16]])
print("A0 row 0 chunk 0 fused:", [round(float(x), 4) for x in vb[0, 0].flatten()[:16]])
for k, (o, w) in REG.items():
    da = (rows_a[:, o:o + w] != rows_b[:, o:o + w])
    db = (rows_b[:, o:o + w] != rows_b2[:, o:o + w])
    rr = torch.nonzero(da.any(1)).flatten().tolist()
    cc = torch.nonzero(da.any(0)).flatten().tolist()
    print(f"{k}: layer!=fused rows {len(rr)} {rr[:12]} cols {len(cc)} {cc[:16]} | fused run-to-run rows "
          f"{int(db.any(1).sum())}")
