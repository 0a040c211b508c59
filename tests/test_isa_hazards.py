"""Static check of the compiled gfx950 code in libvitmi.so for the hazard behind round 2's
misplaced GELU-dropout rows ("SGPR hazard in inline-asm stores"): a VALU instruction
that writes an SGPR (v_readlane / v_readfirstlane, a v_cmp's mask, a carry-out) needs 5 wait
states before a vector-memory instruction reads that SGPR (buffer descriptor, soffset, global
saddr).  hipcc pads the hazard for the instructions it schedules, not for the text of an inline
asm statement; csrc/gemm.hip opens every asm store with `s_nop 4` (VMEM_SGPR_GUARD).  This test
disassembles every device code object and walks each kernel in program order: every instruction
counts one wait state, `s_nop N` N + 1.  Linear order stands in for control flow (a block reached
by a branch is checked against its textual predecessor).  CPU only."""
import glob
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "transformer-stm_amd", "vitmi", "libvitmi.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
WAIT_STATES = 5

_SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b|\b(vcc)\b")
# VALU forms whose SGPR operand(s) in these positions are written
_DST_FIRST = re.compile(r"^v_(readlane|readfirstlane|cmp|cmpx)_")
_DST_SECOND = re.compile(r"^v_(add_co|sub_co|subrev_co|addc_co|subb_co|subbrev_co|mad_u64_u32|mad_i64_i32|div_scale)")
_VMEM = re.compile(r"^(buffer_|global_|scratch_|tbuffer_)")


def _regs(op):
    out = set()
    for m in _SREG.finditer(op):
        if m.group(4):
            out.update(("vcc_lo", "vcc_hi"))
        elif m.group(3) is not None:
            out.add(f"s{m.group(3)}")
        else:
            out.update(f"s{i}" for i in range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def _operands(rest):
    return [o.strip() for o in rest.split("//")[0].split(",")]


def scan(lines):
    """-> list of (kernel, line, text, wait states since the VALU write, sgpr)."""
    bad = []
    kernel, last_write, ws = "?", {}, 0
    for ln in lines:
        m = re.match(r"^[0-9a-f]+ <(.+)>:", ln)
        if m:
            kernel, last_write, ws = m.group(1), {}, 0
            continue
        t = ln.strip()
        if not t or t.startswith(("//", ";")) or t.endswith(":"):
            continue
        t = t.split("//")[0].strip()
        op, _, rest = t.partition(" ")
        ops = _operands(rest) if rest else []
        if _VMEM.match(op):
            for o in ops:
                for r in _regs(o):
                    if r in last_write and ws - last_write[r] < WAIT_STATES:
                        bad.append((kernel, t, ws - last_write[r], r))
        n = 1
        if op == "s_nop":
            n = int(rest.strip(), 0) + 1
        if op.startswith("v_") and ops:
            dsts = []
            if _DST_FIRST.match(op):
                dsts = ops[:1]
            elif _DST_SECOND.match(op) and len(ops) > 1:
                dsts = ops[1:2]
            for d in dsts:
                for r in _regs(d):
                    last_write[r] = ws + 1     # counted from the instruction after the write
        ws += n
    return bad


def test_scanner_flags_a_short_gap_and_accepts_the_guard():
    bad = scan(["0000000000000000 <k>:",
                "\tv_readlane_b32 s53, v1, 0",
                "\tbuffer_store_dwordx4 v[0:3], v5, s[40:43], s53 offen"])
    assert bad and bad[0][3] == "s53"
    ok = scan(["0000000000000000 <k>:",
               "\tv_readlane_b32 s53, v1, 0",
               "\ts_nop 4",
               "\tbuffer_store_dwordx4 v[0:3], v5, s[40:43], s53 offen"])
    assert ok == []


def test_no_valu_sgpr_write_feeds_vmem_within_5_wait_states(tmp_path):
    if not (os.path.exists(OBJDUMP) and os.path.exists(LIB)):
        pytest.skip("needs llvm-objdump and the built library")
    lib = tmp_path / "libvitmi.so"
    shutil.copy(LIB, lib)
    # --offloading extracts the device code objects next to the input file
    subprocess.run([OBJDUMP, "--offloading", str(lib)], check=True, capture_output=True, timeout=120)
    objs = [f for f in glob.glob(str(tmp_path / "libvitmi.so.*")) if "amdgcn" in f]
    assert objs, "no gfx950 code object in the library"
    bad = []
    for f in objs:
        asm = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", f], check=True, capture_output=True,
                             text=True, timeout=300).stdout
        assert "buffer_" in asm or "global_" in asm or len(objs) > 1
        bad += scan(asm.splitlines())
    assert not bad, "VALU-written SGPR read by VMEM too early:\n" + "\n".join(
        f"{k[:60]}: {t} ({w} wait states, {r})" for k, t, w, r in bad[:20])


# ------------------------------------------------------------------ inline-asm loads
# The persistent dK/dV kernels (csrc/attention.hip attn_bwd_dkv_seq_bf16) load K, V, lse and delta
# with inline-asm buffer loads the compiler does not track (asm_load16 / asm_load4) and stage Q | dO
# with inline-asm LDS-DMA (dma_piece, which writes M0).  Correctness rests on the compiled code never
# touching such a load's destination VGPRs before the kernel's own `s_waitcnt vmcnt` (a spill, copy
# or back-edge move would read stale data or be overwritten when the load lands), and on every LDS-DMA
# reading the M0 its own statement just wrote.
_VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def _vregs(text):
    out = set()
    for m in _VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def scan_asm_loads(lines, kernel_filter=lambda k: True):
    """-> list of (kernel, problem): VGPR destinations of a (non-LDS) buffer load referenced before
    the next s_waitcnt vmcnt; an LDS-DMA load not directly preceded (s_nop aside) by its own
    s_mov_b32 m0."""
    bad = []
    kernel, pending, prev = "?", {}, []
    for ln in lines:
        m = re.match(r"^[0-9a-f]+ <(.+)>:", ln)
        if m:
            kernel, pending, prev = m.group(1), {}, []
            continue
        if not kernel_filter(kernel):
            continue
        t = ln.strip().split("//")[0].strip()
        if not t or t.endswith(":"):
            continue
        op, _, rest = t.partition(" ")
        if op == "s_waitcnt" and "vmcnt" in rest:
            pending = {}
        elif op.startswith("buffer_load") and rest.rstrip().endswith(" lds"):
            real = [p for p in prev if not p.startswith("s_nop")]
            if not real or not real[-1].startswith("s_mov_b32 m0,"):
                bad.append((kernel, f"LDS-DMA without its own M0 write: {t}"))
        elif op.startswith(("buffer_load", "global_load")):
            ops = _operands(rest)
            used = _vregs(" ".join(ops[1:]))
            hit = used & set(pending)
            if hit:
                bad.append((kernel, f"{t} uses v{min(hit)} loaded by `{pending[min(hit)]}` before a vmcnt wait"))
            for r in _vregs(ops[0]):
                pending[r] = t
        else:
            hit = _vregs(rest) & set(pending)
            if hit:
                bad.append((kernel, f"{t} touches v{min(hit)} loaded by `{pending[min(hit)]}` before a vmcnt wait"))
        prev = (prev + [t])[-4:]
    return bad


def test_asm_load_scanner_catches_both_hazards():
    lines = ["0000000000000000 <k>:",
             "\tbuffer_load_dwordx4 v[10:13], v2, s[4:7], 0 offen",
             "\tv_mov_b32 v40, v11",
             "\ts_waitcnt vmcnt(0)",
             "\tv_mov_b32 v41, v12",
             "\ts_mov_b32 m0, s3",
             "\ts_nop 0",
             "\tbuffer_load_dwordx4 v5, s[8:11], 0 offen lds",
             "\tv_add_u32 v6, v6, v7",
             "\tbuffer_load_dwordx4 v5, s[8:11], 0 offen lds"]
    bad = scan_asm_loads(lines)
    assert len(bad) == 2 and "v11" in bad[0][1] and "M0" in bad[1][1]


@pytest.mark.parametrize("kern", ["attn_bwd_dkv_seq_bf16", "attn_bwd_fused_seq_bf16"])
def test_dkv_kernels_asm_loads_and_m0(tmp_path, kern):
    """The persistent dK/dV kernels and the persistent single-pass backward (round 6: the next
    pair's Q | dO by dma_piece, its K / V / O rows and lse by asm_load16 / asm_load4)."""
    if not (os.path.exists(OBJDUMP) and os.path.exists(LIB)):
        pytest.skip("needs llvm-objdump and the built library")
    lib = tmp_path / "libvitmi.so"
    shutil.copy(LIB, lib)
    subprocess.run([OBJDUMP, "--offloading", str(lib)], check=True, capture_output=True, timeout=120)
    objs = [f for f in glob.glob(str(tmp_path / "libvitmi.so.*")) if "amdgcn" in f]
    seen, bad = 0, []
    for f in objs:
        asm = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", f], check=True, capture_output=True,
                             text=True, timeout=300).stdout
        if kern not in asm:
            continue
        seen += 1
        bad += scan_asm_loads(asm.splitlines(), lambda k: kern in k)
    assert seen, f"no code object holds {kern}"
    assert not bad, "\n".join(f"{k[:50]}: {p}" for k, p in bad[:20])
