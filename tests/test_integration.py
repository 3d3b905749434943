"""Drop-in boundary: the fhe_common.py backend switch, the optional-symbol fallback
contract (bg:446-462) and host-array validation.  CPU only; none of these touch the GPU."""
import os
import shutil
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
PYDIR = REPO / "fhe-spear_amd" / "python"
REF_FC = Path("/root/reference/fhe_common.py")


@pytest.mark.skipif(not REF_FC.is_file(), reason="reference checkout absent (GPU box)")
def test_fhe_common_patch_selects_mi355x_backend(tmp_path):
    """integration/fhe_common.patch applied to a scratch copy of the reference's fhe_common.py:
    with FHESPEAR_PYPHANTOM pointing at fhe-spear_amd/python, `import pyPhantom` inside
    fhe_common resolves to this repo's module and USE_PHANTOM_GPU is True (fc:9-17)."""
    shutil.copy(REF_FC, tmp_path / "fhe_common.py")
    r = subprocess.run(["patch", "-p1", "-i", str(REPO / "integration" / "fhe_common.patch")], cwd=tmp_path,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    code = ("import sys; sys.dont_write_bytecode = True; sys.path.insert(0, sys.argv[1]); import fhe_common; "
            "import pyPhantom; print(fhe_common.USE_PHANTOM_GPU); print(pyPhantom.__file__)")
    env = dict(os.environ, FHESPEAR_PYPHANTOM=str(PYDIR), PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-c", code, str(tmp_path)], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    use_gpu, path = r.stdout.strip().splitlines()[-2:]
    assert use_gpu == "True"
    assert Path(path).resolve().is_relative_to(PYDIR.resolve())


def test_missing_optional_symbols_raise_attribute_error():
    """A library without a fork-only symbol (simulated with FHESPEAR_DISABLE_SYMBOLS) still imports;
    the matching pyPhantom names are absent, so the reference's try/except AttributeError fallbacks
    (bg:449-452 bsgs_from_cpu -> upload_plaintexts, bg:458-462 bsgs_multiply_accumulate -> loop)
    are taken.  Required symbols stay present."""
    code = r'''
import sys
sys.path.insert(0, sys.argv[1])
import pyPhantom as ph
for name in ("bsgs_from_cpu", "bsgs_complete_from_cpu", "bsgs_multiply_accumulate"):
    try:
        getattr(ph, name)
        print(name, "present")
    except AttributeError:
        print(name, "AttributeError")
print("encode_double_vector_batch", hasattr(ph.ckks_encoder, "encode_double_vector_batch"))
print("rotate", hasattr(ph, "rotate"), "upload_plaintexts", hasattr(ph, "upload_plaintexts"))
'''
    env = dict(os.environ, FHESPEAR_DISABLE_SYMBOLS="fhs_bsgs_from_cpu,fhs_bsgs_multiply_accumulate,"
                                                     "fhs_encode_real_batch")
    r = subprocess.run([sys.executable, "-c", code, str(PYDIR)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    out = r.stdout
    assert "bsgs_from_cpu AttributeError" in out
    assert "bsgs_complete_from_cpu AttributeError" in out
    assert "bsgs_multiply_accumulate AttributeError" in out
    assert "encode_double_vector_batch False" in out
    assert "rotate True upload_plaintexts True" in out


def test_host_diagonal_arrays_are_validated():
    """bsgs_from_cpu / upload_plaintexts check the (count, limbs, N) host array against the context
    before the DMA reads count x limbs x N words."""
    sys.path.insert(0, str(PYDIR))
    import pyPhantom as ph

    class Ctx:
        L0, N = 6, 64
    ctx = Ctx()
    ok = np.zeros((4, 6, 64), dtype=np.uint64)           # chain index 1 -> 6 limbs
    assert ph._host_diagonals(ctx, ok, 1, 6, 64, 4, "t").shape == (4, 6, 64)
    assert ph._host_diagonals(ctx, ok[:, 1:], 2, 5, 64, 3, "t").shape == (4, 5, 64)
    bad = [
        (ok[0], 1, 6, 64, 1),                  # 2-D
        (ok, 2, 6, 64, 4),                     # chain index says 5 limbs
        (ok, 1, 5, 64, 4),                     # coeff_modulus_size mismatch
        (ok, 1, 6, 32, 4),                     # poly_modulus_degree mismatch
        (ok[:, :, :32], 1, 6, 64, 4),          # array narrower than N
        (ok, 1, 6, 64, 5),                     # fewer plaintexts than D
    ]
    for a, ci, cms, pmd, cnt in bad:
        with pytest.raises(ValueError):
            ph._host_diagonals(ctx, a, ci, cms, pmd, cnt, "t")
