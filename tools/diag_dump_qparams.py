import sys, torch
sys.path.insert(0, ".")
from quantized_vit_amd.calibrate import build_quantized_vit
m = build_quantized_vit("vit_large_patch16_384", seed=0, device=torch.device("cuda"))
sd = {k: v.detach().cpu() for k, v in m.state_dict().items() if ("quant" in k or "q_m" in k)}
import os; os.makedirs("gpurun_out/r04c", exist_ok=True)
torch.save(sd, "gpurun_out/r04c/vitl_qparams.pt")
print(len(sd))
