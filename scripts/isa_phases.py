"""Static instruction mix of one kernel, attributed to the source function it
came from (line tables + inline stacks), e.g. the fused unicycle step's
phases: pre-step sincos, get_state, CBF rows, QP (per wave-uniform KK
branch and stage), env step, observation, stores.

Build the TU with line tables (device only) first, e.g.
  hipcc <the build's HIP_FLAGS> -gline-tables-only --cuda-device-only -c -o env_g.co csrc/rcbf_env.hip
  clang-offload-bundler --unbundle --type=o --input=env_g.co \
      --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=env_g.elf
then
  python scripts/isa_phases.py env_g.elf k_safe_stepILi0ELi1ELi5ELb0ELi256ELb0E [--paths]

Counts are static (each instruction once); the kernel's dynamic VALU per
wave (SQ_INSTS_VALU / SQ_WAVES, scripts/pmc_sq.py) is the other half of the
picture: a wave runs one KK branch of the QP and skips the reset path unless
one of its envs resets.
"""
import re
import subprocess
import sys
from collections import Counter, defaultdict

LLVM = "/opt/rocm/lib/llvm/bin"
# generic math / intrinsic wrappers: attributed to their caller
GENERIC = {"fma", "fmax", "fmin", "fabs", "fabsf", "sqrt", "rint", "isfinite", "copysign", "__builtin_copysign",
           "rcp64_nz", "rcp64_qp_nz", "operator()", "__ballot", "__popc", "__shfl", "__shfl_xor", "max", "min"}


def base(fn):
    fn = re.sub(r"\(.*", "", fn)  # drop the argument list (and everything after it)
    depth, out = 0, []
    for ch in fn:  # drop template arguments
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif depth == 0:
            out.append(ch)
    s = "".join(out).strip()
    return s.split("::")[-1].split()[-1] if s else fn


def kk_of(fn):
    m = re.search(r"uni_slots_solve<(\d+)", fn) or re.search(r"uni_pieces_solve<(\d+)", fn)
    return int(m.group(1)) if m else None


def disasm(elf, sym_sub):
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", elf], capture_output=True,
                         text=True, check=True).stdout
    ins, on = [], False
    for line in out.splitlines():
        if re.match(r"^[0-9a-f]+ <.*>:$", line):
            on = sym_sub in line
            continue
        if not on:
            continue
        m = re.match(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):", line)
        if m:
            ins.append((int(m.group(3), 16), m.group(1)))
    return ins


def symbolize(elf, addrs):
    inp = "\n".join("0x%x" % a for a in addrs) + "\n"
    out = subprocess.run([f"{LLVM}/llvm-symbolizer", "--obj=" + elf, "--inlines", "--functions=linkage",
                          "--demangle"], input=inp, capture_output=True, text=True, check=True).stdout
    blocks = out.strip("\n").split("\n\n")
    stacks = []
    for b in blocks:
        lines = b.splitlines()
        frames = [(lines[k], lines[k + 1]) for k in range(0, len(lines) - 1, 2)]
        stacks.append(frames[::-1])  # outermost first
    return stacks


def stage_lines():
    """Line numbers of the stage markers in uni_pieces_solve (rcbf_device.hpp)."""
    import os
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sac-rcbf_amd", "csrc", "rcbf_device.hpp")
    marks = {}
    for n, line in enumerate(open(src), 1):
        for key in ("// stage 1b:", "// stage 2:"):
            if key in line and key not in marks:
                marks[key] = n
    return marks["// stage 1b:"], marks["// stage 2:"]


STAGE_1B, STAGE_2 = stage_lines()


def phase_of(frames):
    names = [f for f, _ in frames]
    bases = [base(f) for f in names]
    if "safe_step_one" not in bases:
        inner = [b for b in bases[1:] if b not in GENERIC]
        return "kernel: " + (inner[0] if inner else "loads, addresses, stores, control")
    i = bases.index("safe_step_one")
    inner = [(b, n, ln) for b, n, ln in zip(bases[i + 1:], names[i + 1:], [l for _, l in frames[i + 1:]])
             if b not in GENERIC]
    if not inner:
        return "safe_step_one glue"
    b0 = inner[0][0]
    if b0 == "sincos":
        return "pre-step sincos(theta), fp64"
    if b0 == "layer_forward":
        bs = [b for b, _, _ in inner]
        kk = next((kk_of(n) for _, n, _ in inner if kk_of(n)), None)
        if "uni_pieces_solve" in bs:
            line = int(inner[bs.index("uni_pieces_solve")][2].rsplit(":", 2)[-2])
            stage = "1a origin + pieces" if line < STAGE_1B else ("1b kinks + triples" if line < STAGE_2 else "2 edges")
            return f"QP KK = {kk}: stage {stage}"
        if "uni_slots_solve" in bs:
            return f"QP KK = {kk}: slot compaction, eps"
        if "uni_qp_2d_core" in bs or "wave_max_count" in bs:
            return "QP live-row test, wave KK, status"
        if "uni_rows_diff_cs" in bs:
            return "CBF rows (fp32)"
        return "layer: raw rows in, clamp out"
    return {"uni_state32_from_cs": "get_state (theta32 from cos/sin)", "uni_env_step_cs": "env step",
            "env_reset_one": "auto-reset"}.get(b0, b0)


def main():
    elf, sym = sys.argv[1], sys.argv[2]
    ins = disasm(elf, sym)
    if not ins:
        sys.exit("kernel not found")
    stacks = symbolize(elf, [a for a, _ in ins])
    assert len(stacks) == len(ins), (len(stacks), len(ins))
    rows = defaultdict(Counter)
    paths = Counter()
    for (a, op), fr in zip(ins, stacks):
        ph = phase_of(fr)
        c = rows[ph]
        c["all"] += 1
        if op.startswith("v_"):
            c["valu"] += 1
            if "f64" in op:
                c["valu_f64"] += 1
            if op.startswith(("v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos", "v_exp", "v_log")):
                c["trans"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            c["vmem"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        if "--paths" in sys.argv:
            paths[" > ".join(base(f) for f, _ in fr)] += 1
    tot = Counter()
    print(f"{'phase':58s} {'instr':>6s} {'VALU':>6s} {'f64':>6s} {'trans':>6s} {'VMEM':>5s} {'LDS':>4s} {'SALU':>5s}")
    for ph, c in sorted(rows.items(), key=lambda kv: -kv[1]["valu"]):
        tot.update(c)
        print(f"{ph[:58]:58s} {c['all']:6d} {c['valu']:6d} {c['valu_f64']:6d} {c['trans']:6d} {c['vmem']:5d} "
              f"{c['lds']:4d} {c['salu']:5d}")
    print(f"{'total':58s} {tot['all']:6d} {tot['valu']:6d} {tot['valu_f64']:6d} {tot['trans']:6d} {tot['vmem']:5d} "
          f"{tot['lds']:4d} {tot['salu']:5d}")
    if "--paths" in sys.argv:
        for p, n in paths.most_common(60):
            print(n, p)


if __name__ == "__main__":
    main()
