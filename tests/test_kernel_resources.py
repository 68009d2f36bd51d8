"""Register / scratch guard for the built engine (CPU: reads the gfx950 code objects inside
libvap_hip.so, no GPU).

Round 4 found every gemm2_kernel instantiation spilling 64-84 VGPRs into 148-180 B of scratch per
lane (a runtime branch over 128 live accumulators): scratch is HBM traffic and its
reloads' vmcnt(0) serialises the epilogue, yet nothing failed.  This test reads each kernel's
metadata (``.private_segment_fixed_size``, ``.vgpr_spill_count``) from the code objects of the
library's offload bundles and fails on any scratch in a production kernel.  Allowed: the
stamp-diagnostic instantiations (VAP_*_STAMPS builds) and the 144-row block kernel, which the engine
never selects (launch_block is always called with cus = 0).
"""
import os
import re
import shutil
import struct
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "voiceactivityprojection_amd", "_lib", "libvap_hip.so")
READOBJ = "/opt/rocm/lib/llvm/bin/llvm-readobj"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# (name regex, reason): kernels allowed to use scratch
ALLOWED = [
    (r"conv01m_kernelILb1E", "stamp-diagnostic build (VAP_CONV01_STAMPS)"),
    (r"convk4_kernelILi16E", "debug-mode build (VAP_CONVK4_DBG)"),
    (r"block_kernelILi9E", "144-row variant, not selected by the engine"),
]


def _fatbin(path: str) -> bytes:
    if not shutil.which("objcopy"):
        pytest.skip("objcopy not available")
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "fat.bin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, out], check=True)
        with open(out, "rb") as f:
            return f.read()


def _code_objects(fat: bytes):
    """gfx950 code objects of every offload bundle in the section (one bundle per linked object)."""
    pos = 0
    while True:
        i = fat.find(MAGIC, pos)
        if i < 0:
            return
        n = struct.unpack_from("<Q", fat, i + len(MAGIC))[0]
        p = i + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple and size:
                yield fat[i + off:i + off + size]
        pos = i + len(MAGIC)


def _kernel_meta(code: bytes):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(code)
        f.flush()
        txt = subprocess.run([READOBJ, "--notes", f.name], check=True, capture_output=True, text=True).stdout
    for blk in txt.split(".name:")[1:]:
        name = blk.split("\n")[0].strip()

        def g(key):
            m = re.search(r"\." + key + r":\s+(\d+)", blk)
            return int(m.group(1)) if m else 0

        yield name, g("private_segment_fixed_size"), g("vgpr_spill_count"), g("sgpr_spill_count")


def test_no_scratch_in_production_kernels():
    if not os.path.exists(LIB):
        pytest.skip("library not built (python -c 'import __graft_entry__ as g; g.build()')")
    if not os.path.exists(READOBJ):
        pytest.skip("llvm-readobj not available")
    kernels = [k for co in _code_objects(_fatbin(LIB)) for k in _kernel_meta(co)]
    assert len(kernels) > 40, f"found only {len(kernels)} kernels in the library's code objects"
    names = {k[0] for k in kernels}
    for must in ("lstm_pair_kernel", "conv01m_kernel", "attn4_kernel", "block_kernel", "gemm2_kernel",
                 "gemm3_kernel", "lstm_quad_kernel"):
        assert any(must in n for n in names), f"{must} missing from the code objects"
    bad = []
    for name, priv, vspill, sspill in kernels:
        if priv == 0 and vspill == 0 and sspill == 0:
            continue
        if any(re.search(rx, name) for rx, _ in ALLOWED):
            continue
        bad.append(f"{name}: scratch {priv} B, VGPR spills {vspill}, SGPR spills {sspill}")
    assert not bad, "production kernels with scratch:\n" + "\n".join(bad)
