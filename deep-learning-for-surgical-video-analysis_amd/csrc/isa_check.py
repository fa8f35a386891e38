"""Build-time audit of the gfx950 code objects in the svk objects (run by the Makefile after linking).

1. Packed-FP32 VALU ops.  On gfx950 a VALU write of a VGPR followed by a v_pk_*_f32 that reads it as the
   LOW lane's source through op_sel (e.g. ``v_pk_add_f32 v[0:1], v[42:43], v[44:45] op_sel:[0,1]``) reads
   stale data in lanes 48-63 while another wave of the same SIMD issues MFMAs; s_nop 1 does not cover it
   and hipcc 7.2 inserts no wait (reproduced by tools/hazard/pk_hazard.hip: 1.5 % of lanes 48-63 wrong
   under MFMA load, none without op_sel or without the load; it was the round-2 gemm_pk "stale epilogue
   element").  The library is built without packed-FP32 ops; this check proves no such instruction
   (v_pk_add/mul/fma_f32, or v_pk_mov_b32 with op_sel) reached the code objects.  Also rejected:
   v_ashr_pk_u8_i32 / v_ashr_pk_i8_i32, which hipcc 7.2 emits for two shift-clamp-pack chains assuming the
   upper 16 destination bits are zeroed; on the GPU they keep the register's old contents (augment.hip's
   vertical pass produced OR-ed bytes until it blocked the fusion).
2. Epilogue operand loads of gemm_pk.  They are issued from inline asm so hipcc's waitcnt pass does not
   drain the cross-tile LDS-DMA prefetch; their completion is covered by the counted vmcnt of the tile's
   last K-step.  hipcc treats the destination VGPRs as written when the asm statement ends, so any
   compiler instruction touching them before that wait would read or clobber in-flight data.  Every
   VGPR-destination global_load in a gemm_pk kernel is followed, on EVERY control-flow path, by an
   s_waitcnt with a vmcnt field before any instruction reads or writes its destination registers.  The same
   holds for dwfc2_rw (round 5: its K-loop W2 / tap loads are asm too; a runtime index into a double
   buffer of such registers once made hipcc copy them right after the load, the copy read in-flight data
   and a reused address register was overwritten by the returning load — the GPU hung).
Exit status 1 with a report on any violation."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
INS_RE = re.compile(r"^\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-F]+):")
TGT_RE = re.compile(r"<([A-Za-z0-9_.$]+)\+0x([0-9a-f]+)>")
SYM_RE = re.compile(r"^([0-9a-f]+) <([^>]+)>:")


def regs(tok):
    tok = tok.strip()
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def disasm(obj, notes_out=None):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "g.co")
        r = subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", obj,
                            os.path.join(d, "o")], capture_output=True)
        if r.returncode != 0 or not os.path.exists(fat):
            return ""                                          # host-only object: no device code
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--targets={TARGET}",
                        f"--input={fat}", f"--output={co}"], check=True, capture_output=True)
        if notes_out is not None:
            notes_out.append(subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                            text=True).stdout)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                              capture_output=True, text=True).stdout


def functions(text):
    """{symbol: [(addr, op, operands, branch_target_addr_or_None)]}"""
    funcs, cur, base = {}, None, 0
    for line in text.split("\n"):
        m = SYM_RE.match(line)
        if m:
            cur, base = m.group(2), int(m.group(1), 16)
            funcs[cur] = []
            continue
        m = INS_RE.match(line)
        if m and cur is not None:
            t = TGT_RE.search(line)
            tgt = base + int(t.group(2), 16) if (t and t.group(1) == cur) else None
            funcs[cur].append((int(m.group(3), 16), m.group(1), m.group(2), tgt))
    return funcs


def operands(s):
    parts = [p.strip() for p in s.split(",")]
    return [p.split()[0] for p in parts if p]


def check_packed(funcs):
    bad = []
    for f, ins in funcs.items():
        for addr, op, ops, _ in ins:
            # packed f32 arithmetic is allowed only with the default op_sel (the hand-written svk_common.h pk_*
            # helpers): the gfx950 hazard needs a low lane read THROUGH op_sel (tools/hazard/pk_hazard.hip)
            if (re.match(r"v_pk_(add|mul|fma)_f32", op) and "op_sel" in ops) or (op == "v_pk_mov_b32" and "op_sel" in ops):
                bad.append(f"{f}+0x{addr:x}: {op} {ops}")
            if re.match(r"v_ashr_pk_[iu]8_i32", op):
                bad.append(f"{f}+0x{addr:x}: {op} {ops} (16-bit result, upper half kept by the hardware)")
    return bad


VMEM_RE = re.compile(r"(global_|buffer_|flat_|scratch_)")
ASM_LOAD_KERNELS = ("gemm_pk", "dwfc2_rw", "gemm_ln")          # kernels whose global loads are issued from inline asm
VMCNT_RE = re.compile(r"vmcnt\((\d+)\)")
LOAD_RE = re.compile(r"global_load_(dword(x2|x4)?|ushort|ubyte|short_d16|sshort)$")   # VGPR-destination loads


def check_epilogue_loads(funcs):
    """For every VGPR-destination global_load of a gemm_pk kernel, on every control-flow path: the first
    s_waitcnt vmcnt(n) with at least n vector-memory operations issued after the load (so the load is not
    among the n youngest and has retired) comes before any instruction reading or writing its
    destination registers."""
    bad = []
    for f, ins in funcs.items():
        if not any(t in f for t in ASM_LOAD_KERNELS):
            continue
        at = {a: k for k, (a, *_rest) in enumerate(ins)}
        for k, (addr, op, ops, _) in enumerate(ins):
            if not LOAD_RE.match(op):
                continue
            dst = regs(operands(ops)[0])
            seen, stack = {}, [(k + 1, 0, None)]
            while stack:
                j, younger, prev = stack.pop()
                if j >= len(ins):
                    continue
                # the path with the FEWEST younger operations is the one a wait may fail to cover: a visit
                # with at least as many as an earlier one is dominated
                if j in seen and seen[j] <= younger:
                    continue
                seen[j] = younger
                key = j
                a2, op2, ops2, tgt = ins[j]
                if op2 == "s_waitcnt":
                    m = VMCNT_RE.search(ops2)
                    if m and younger >= int(m.group(1)):
                        continue                              # retired on this path
                touched = set()
                for o in operands(ops2):
                    touched |= regs(o)
                if op2.startswith(("v_", "global_", "ds_", "buffer_", "flat_")) and touched & dst:
                    bad.append(f"{f}+0x{addr:x}: {op} {ops} -> touched at +0x{a2:x}: {op2} {ops2}")
                    continue
                if VMEM_RE.match(op2):
                    younger += 1
                if op2 == "s_endpgm":
                    continue
                if op2 == "s_branch":
                    stack.append((at.get(tgt, len(ins)), younger, key))
                    continue
                if op2.startswith("s_cbranch") and tgt is not None:
                    stack.append((at.get(tgt, len(ins)), younger, key))
                stack.append((j + 1, younger, key))
    return bad


def check_scratch(notes):
    """gemm_pk / gemm_pp kernels must not use scratch (a spill of a register an inline-asm load is still writing
    would store garbage; the round-3 256x256 tile that spilled faulted the GPU; and a scratch access is a vector
    memory operation that the hand-counted `s_waitcnt vmcnt(N)` of the LDS-DMA pipelines does not know about)."""
    bad, cur = [], None
    for line in notes.split("\n"):
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            cur = m.group(1)
        m = re.match(r"\s+\.(private_segment_fixed_size|vgpr_spill_count):\s+(\d+)", line)
        if m and int(m.group(2)) > 0 and cur and any(t in cur for t in ASM_LOAD_KERNELS + ("gemm_pp",)):
            bad.append(f"{cur}: .{m.group(1)} {m.group(2)}")
    return bad


def main(objs):
    fails = 0
    nload = 0
    for obj in objs:
        notes = []
        funcs = functions(disasm(obj, notes))
        for msg in check_scratch(notes[0] if notes else ""):
            print(f"isa_check: {os.path.basename(obj)}: scratch use in a kernel with inline-asm loads: {msg}")
            fails += 1
        for msg in check_packed(funcs):
            print(f"isa_check: {os.path.basename(obj)}: packed-FP32 op_sel hazard class: {msg}")
            fails += 1
        for msg in check_epilogue_loads(funcs):
            print(f"isa_check: {os.path.basename(obj)}: epilogue load register touched before its wait: {msg}")
            fails += 1
        nload += sum(1 for f, ins in funcs.items() if any(t in f for t in ASM_LOAD_KERNELS) for _, op, _, _ in ins
                     if LOAD_RE.match(op))
    print(f"isa_check: {len(objs)} objects, {nload} asm-load kernel loads audited ({', '.join(ASM_LOAD_KERNELS)}), "
          f"{fails} violation(s)")
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
