"""Does torch's HIP init work after libfhespear_hip initialised HIP (and after an OOM)?"""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "fhe-spear_amd" / "python"))
import pyPhantom as ph

mode = sys.argv[1]
N = 16384
parms = ph.params(ph.scheme_type.ckks)
parms.set_poly_modulus_degree(N)
parms.set_special_modulus_size(3)
parms.set_galois_elts([ph.get_elt_from_step(1, N)])
parms.set_coeff_modulus(ph.create_coeff_modulus(N, [59] * 39))
ctx = ph.context(parms)
if mode == "oom":
    try:
        ph.random_plaintexts(ctx, 3, 70000, 1, 2.0 ** 59)
    except RuntimeError as e:
        print("oom:", e)
import torch
print("torch device_count", torch.cuda.device_count(), flush=True)
print("mem_get_info", torch.cuda.mem_get_info(0), flush=True)
