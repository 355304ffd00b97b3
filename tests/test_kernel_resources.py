"""Every gfx950 kernel in libsnakehip.so runs out of registers (CPU, no GPU).

Round 3 shipped syrk_h3q_kernel with two stage lambdas the compiler did not
inline: their captured fragments went to scratch and D(16k) took 3.2 s instead
of ~60 ms, with every parity test still green. A scratch or spill regression is
a performance bug that no numeric test sees, so this test reads the kernel
descriptors' metadata straight out of the built library:

  - the .hip_fatbin section holds one clang offload bundle per translation
    unit; each bundle's `hipv4-amdgcn-amd-amdhsa--gfx950` entry is an ELF code
    object;
  - `llvm-readelf --notes` prints that object's AMDGPU metadata, one block per
    kernel with .private_segment_fixed_size (scratch bytes per lane),
    .vgpr_spill_count and .sgpr_spill_count.

Every kernel must report no scratch and no VGPR spills, and the hot-path
kernels named below must be present (a renamed or dropped kernel would
otherwise pass silently). SGPR spills are allowed: they go to VGPR lanes
(v_writelane), not to memory, and scratch 0 proves it.
"""
import os
import re
import struct
import subprocess

import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
LIB = os.path.join(REPO, "laplace-dqn-snake-game_amd", "libsnakehip.so")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# (substring of the mangled name, what it is) -- the kernels bench.py times
HOT = [
    ("syrk_h3k_kernel", "Jacobian Gram D(n): conv sections, 256 x 256 tiles, K-split fp32 partials"),
    ("syrk_ksum_kernel", "Jacobian Gram D(n): fp64 chunk sum + Dense terms + mirror"),
    ("syrk_h3q_kernel", "Jacobian Gram D(n): DENSE sections (and the round-5 conv kernel)"),
    ("h3_seg_rows_kernel", "Dense-section h3 operand split"),
    ("syrk_slab_kernel", "snapshot Gram D'D (fp64 slabs)"),
    ("conv_h3f", "per-sample Jacobian rows (fp32-faithful conv)"),
    ("grad_update_kernel", "RMSProp + target copy + next replay draw"),
    ("upd_fwd", "update forward"),
    ("replay_sample_wave_kernel", "replay draw"),
]


def code_objects(path: str):
    """Yield the gfx950 ELF images inside the fat binary."""
    data = open(path, "rb").read()
    start = 0
    while (s := data.find(MAGIC, start)) >= 0:
        n, = struct.unpack_from("<Q", data, s + len(MAGIC))
        p = s + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tlen].decode()
            p += tlen
            if "gfx950" in triple and size:
                yield data[s + off:s + off + size]
        start = s + len(MAGIC)


def kernel_metadata(path: str, tmp) -> dict:
    """mangled name -> {field: int} for every kernel in every code object."""
    out = {}
    for i, elf in enumerate(code_objects(path)):
        f = tmp / f"co{i}.elf"
        f.write_bytes(elf)
        notes = subprocess.run([READELF, "--notes", str(f)], check=True,
                               capture_output=True, text=True).stdout
        # each kernel's block starts at "- .agpr_count" / "- .args" etc.; split on
        # the .name line and read the numeric fields of the block around it
        blocks = re.split(r"\n\s+- \.", notes)
        for b in blocks:
            m = re.search(r"\.name:\s+(\S+)", b)
            if not m or ".kernarg_segment_size" not in b:
                continue
            fields = {k: int(v) for k, v in re.findall(
                r"\.(private_segment_fixed_size|vgpr_spill_count|sgpr_spill_count|vgpr_count|agpr_count):\s+(\d+)", b)}
            out[m.group(1)] = fields
    return out


@pytest.fixture(scope="module")
def meta(tmp_path_factory):
    if not os.path.exists(READELF):
        pytest.skip("llvm-readelf not in this image")
    if not os.path.exists(LIB):
        pytest.fail("libsnakehip.so is not built (run __graft_entry__.build())")
    return kernel_metadata(LIB, tmp_path_factory.mktemp("co"))


def test_hot_kernels_present(meta):
    assert len(meta) > 100, len(meta)
    for key, what in HOT:
        assert any(key in k for k in meta), f"{what}: no kernel matching {key!r}"


def test_no_kernel_uses_scratch_or_spills(meta):
    bad = []
    for name, f in sorted(meta.items()):
        assert {"private_segment_fixed_size", "vgpr_spill_count", "sgpr_spill_count"} <= f.keys(), name
        if f["private_segment_fixed_size"] or f["vgpr_spill_count"]:
            bad.append((name, f["private_segment_fixed_size"], f["vgpr_spill_count"], f["sgpr_spill_count"]))
    assert not bad, "kernels with scratch/VGPR spills (name, scratch B, vgpr spills, sgpr spills):\n" + \
        "\n".join(map(str, bad))


def test_syrk_h3q_register_budget(meta):
    """The Gram kernels hold 2 waves/SIMD (8 waves/WG, 1 WG/CU):
    arch VGPRs + AGPRs must fit in 256."""
    k = [n for n in meta if "syrk_h3q_kernel" in n or "syrk_h3k_kernel" in n]
    assert any("syrk_h3k_kernel" in n for n in k)
    assert k
    for n in k:
        f = meta[n]
        assert f["vgpr_count"] + f.get("agpr_count", 0) <= 256, (n, f)


def test_no_wrong_result_measurement_variants(meta):
    """The Gram kernel's measurement variants (VAR 1: no MFMA, VAR 2: no stage
    DMAs; wrong results by design) exist only in the measurement build
    (make measure, -DSNK_SYRK_MEASURE): the shipping library holds VAR 0 only,
    so no environment variable can select them."""
    bad = [n for n in meta if re.search(r"syrk_h3q_kernelILi[1-9]E|syrk_h3_kernelILi\d+ELi[1-9]E", n)]
    assert not bad, bad
    assert any(re.search(r"syrk_h3q_kernelILi0E", n) for n in meta)
