"""The hot-column CSR kernel keeps its two gather policies,
checked on the device assembly the shipped object is assembled from.

The first form loaded hot rows with a plain load and cold rows with
__builtin_nontemporal_load in the two arms of a wave-uniform branch; hipcc
merged the arms into one plain load and the nt hint was gone (no error, no
wrong result: only the speed-up). The shipped form uses raw buffer loads whose
cache policy is an immediate, so each instantiation must hold both a
default-policy and an nt B-row buffer load, in equal numbers."""
from __future__ import annotations

import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "spmm-denseblock_amd")
ASM = os.path.join(PKG, "build", "csr_kernels-hip-amdgcn-amd-amdhsa-gfx950.s")


@pytest.fixture(scope="module")
def csr_asm() -> str:
    if not os.path.exists(ASM):
        subprocess.run(["make", "-C", PKG, "lib"], check=True, capture_output=True)
    with open(ASM) as f:
        return f.read()


def _bodies(asm: str, pattern: str) -> dict[str, str]:
    out = {}
    for m in re.finditer(r"^(_Z\S*" + pattern + r"\S*):", asm, re.M):
        end = asm.find(".Lfunc_end", m.end())
        out[m.group(1)] = asm[m.end():end]
    return out


def _hot_mode(name: str) -> int:
    # csr_mergepath_kernel<VEC, NT, HOT>: mangled ...ILi<VEC>ELb<NT>ELi<HOT>EE...
    m = re.search(r"ILi(\d)ELb([01])ELi(\d)EE", name)
    assert m, name
    return int(m.group(3))


def test_hot_kernels_keep_both_policies(csr_asm):
    # HOT = 1 (a resource per row) and HOT = 2 (one resource, the row in soffset)
    hot = {k: v for k, v in _bodies(csr_asm, "csr_mergepath_kernel").items() if _hot_mode(k)}
    assert len(hot) == 6, f"expected VEC 1 / 2 / 4 x HOT 1 / 2 instantiations, found {sorted(hot)}"
    for name, body in hot.items():
        loads = re.findall(r"^\s*buffer_load_dword\S*\s[^\n]*$", body, re.M)
        nt = [ln for ln in loads if re.search(r"\bnt\b", ln)]
        plain = [ln for ln in loads if not re.search(r"\b(nt|sc0|sc1)\b", ln)]
        assert nt and plain, f"{name}: {len(plain)} default-policy / {len(nt)} nt buffer loads"
        assert len(nt) == len(plain), f"{name}: unequal arms {len(plain)} / {len(nt)}"


def test_plain_kernels_have_no_buffer_gathers(csr_asm):
    plain = {k: v for k, v in _bodies(csr_asm, "csr_mergepath_kernel").items()
             if not _hot_mode(k)}
    assert plain
    for name, body in plain.items():
        assert "buffer_load" not in body, f"{name}: the plain kernel changed its gathers"
