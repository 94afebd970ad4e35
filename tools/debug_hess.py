import sys
from pathlib import Path
import numpy as np
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
from golden_util import load
from gpu_util import generator, product_equation, product_module
from oracle import dpi_oracle as O
from golden_util import oracle_equation, oracle_net

f = load("gbm_hess_zero_K2")
eq = product_equation(f)
gen = generator(f, eq, product_module(f, eq))
tx = torch.as_tensor(f["tx"], dtype=torch.float32, device="cuda:0")
y = gen.generate_with_gradients_and_hessians(tx, point_base=int(f["point_base"])).cpu().numpy()
oeq = oracle_equation(f)
onet = oracle_net(f, oeq)
yo, pT, pI = O.labels_grad_hess(oeq, onet, f["tx"], int(f["M"]), int(f["K"]), int(f["seed"]), int(f["epoch"]),
                               int(f["point_base"]), return_parts=True)
nx = 100
H = y[:, 101:].reshape(-1, nx, nx)
HT = pT[:, 101:].reshape(-1, nx, nx)
HI = pI[:, 101:].reshape(-1, nx, nx)
for r in range(2):
    print("point", r)
    print(" gpu diag[:5]", H[r].diagonal()[:5], " off[0,1:4]", H[r][0, 1:4])
    print(" oT  diag[:5]", HT[r].diagonal()[:5], " off", HT[r][0, 1:4])
    print(" oI  diag[:5]", HI[r].diagonal()[:5], " off", HI[r][0, 1:4])
    for name, ref in (("T", HT[r]), ("I", HI[r]), ("T+I", HT[r] + HI[r])):
        print("  rel vs", name, np.linalg.norm(H[r] - ref) / np.linalg.norm(ref))
    print("  sym", np.abs(H[r] - H[r].T).max(), " gpu-ref diag", (H[r] - HT[r] - HI[r]).diagonal()[:4])
np.savez("gpurun_out/dh.npz", y=y, tx=f["tx"])
