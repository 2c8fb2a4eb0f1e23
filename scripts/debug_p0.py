import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "montecarlo-gated-mil_amd"), REPO, os.path.join(REPO, "tests")]
import numpy as np, torch
from golden_util import Case
from mcgmil import ops
case = Case("edge_N200_T3_sep_p0")
dev = torch.device("cuda", 0)
H, _, arrays = case.inputs()
head = ops.HeadTensors(*[torch.from_numpy(np.ascontiguousarray(arrays[k])).to(dev) for k in ops.HeadTensors._fields])
out = ops.mcdo_forward(torch.from_numpy(H).to(dev), ops.bag_offsets_tensor([case.N], dev), head, case.T,
                       p_feat=0.0, p_att=0.0, seed=1, return_stats=True)
A = out["A"].view(case.T, case.C, case.N).cpu().numpy()
Av = out["A_var"].view(case.C, case.N).cpu().numpy()
print("A diff across t:", np.abs(A - A[0:1]).max(), "Av max", np.abs(Av).max(), "argmax", np.unravel_index(np.abs(Av).argmax(), Av.shape))
print("Av nonzero count", (Av != 0).sum(), Av[Av != 0][:10])
print("golden var max", np.abs(case.z["A_var"]).max())
