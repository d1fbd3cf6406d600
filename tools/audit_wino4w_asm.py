"""Audit conv_wino4w's device assembly for the inline-asm accumulator contract (winograd4w.hip,
`mfma_v`): hipcc neither sees nor pads the VGPR accumulators of the asm `v_mfma_f32_16x16x4_f32`
statements, so the build is safe only if, in every conv_wino4w instantiation,

  * no compiler instruction inside the chunk loop (the blocks hipcc annotates `in Loop` / `Loop
    Header`) reads, writes, copies or spills a register that an asm MFMA accumulates into;
  * none does so between the loop exit and the `w4w_drain` nop statement (the 12 wait states an
    8-pass MFMA result needs before another reader);
  * the kernel has no scratch (`.private_segment_fixed_size 0`, `.vgpr_spill_count 0`).

Usage: python tools/audit_wino4w_asm.py [file.s]  (without a file it compiles winograd4w.hip with
hipcc --cuda-device-only -S into a temporary directory). Exit status 1 and one line per finding
when the contract is broken. tests/test_host.py runs it on every CPU test pass.
"""
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(REPO, "fully-automated-multi-heartbeat-echocardiography-video-segmentation-and-motion-tracking_amd",
                   "csrc", "winograd4w.hip")

_VREG = re.compile(r"(?<![\w\[])v(\d+)\b")
_VRANGE = re.compile(r"(?<![\w])v\[(\d+):(\d+)\]")


def regs_of(text):
    """VGPR numbers named in an instruction's text."""
    out = set(int(m) for m in _VREG.findall(text))
    for a, b in _VRANGE.findall(text):
        out.update(range(int(a), int(b) + 1))
    return out


def compile_asm(src=SRC, out_dir=None):
    out_dir = out_dir or tempfile.mkdtemp(prefix="w4w-asm-")
    out = os.path.join(out_dir, "winograd4w.s")
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.join(REPO, "include"),
           "--cuda-device-only", "-S", src, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed ({r.returncode}): {r.stderr[-3000:]}")
    return out


def split_functions(lines):
    """{kernel name: [lines of its body]} for the conv_wino4w kernels (body = from the function
    label to `.Lfunc_end`)."""
    funcs, cur, name = {}, None, None
    for ln in lines:
        m = re.match(r"^(_Z\w*conv_wino4w\w*):", ln)
        if m:
            name, cur = m.group(1), []
            continue
        if cur is not None:
            if ln.startswith(".Lfunc_end"):
                funcs[name] = cur
                cur, name = None, None
            else:
                cur.append(ln)
    return funcs


def audit_function(name, body):
    problems = []
    # asm statements (;;#ASMSTART .. ;;#ASMEND) and the accumulators of their v_mfma, per line
    in_asm = [False] * len(body)
    acc_at = {}  # line -> registers an asm MFMA accumulates into
    i = 0
    while i < len(body):
        if ";;#ASMSTART" in body[i]:
            j = i
            while ";;#ASMEND" not in body[j]:
                in_asm[j] = True
                s = body[j].split(";")[0].strip()
                if s.startswith("v_mfma"):
                    acc_at[j] = regs_of(s.split(None, 1)[1].split(",")[0])
                j += 1
            in_asm[j] = True
            i = j + 1
        else:
            i += 1
    if not acc_at:
        return problems  # an instantiation with no asm MFMAs (NTN <= W4W_NTA)
    # blocks: a label line starts one
    label = None
    in_loop = [False] * len(body)
    for k, ln in enumerate(body):
        if re.match(r"^\.LBB\w+:", ln):
            label = ln
        in_loop[k] = label is not None and "Loop" in label
    # each chunk loop (a run of loop blocks; the two-item form has two, with their own register
    # assignment) is checked against the accumulators of ITS asm MFMAs, together with its exit prefix:
    # from the loop's last line to the next drain statement
    k = 0
    while k < len(body):
        if not in_loop[k]:
            k += 1
            continue
        b = k
        e = k
        while e + 1 < len(body) and in_loop[e + 1]:
            e += 1
        acc = set().union(*[r for ln, r in acc_at.items() if b <= ln <= e]) if any(b <= ln <= e for ln in acc_at) else set()
        k = e + 1
        if not acc:
            continue  # a loop without asm MFMAs
        drain = next((d for d in range(e + 1, len(body)) if in_asm[d] and "s_nop 7" in body[d]), None)
        if drain is None:
            problems.append(f"{name}: no w4w_drain nop statement after the chunk loop ending at line {e}")
            drain = e + 1
        for x in range(b, drain):
            if in_asm[x]:
                continue
            s = body[x].split(";")[0].strip()
            if not s or s.endswith(":") or s.startswith("."):
                continue
            hit = regs_of(s) & acc
            if hit:
                where = "chunk loop" if in_loop[x] else "loop exit before the drain"
                problems.append(f"{name}: compiler instruction in the {where} touches asm accumulator "
                                f"v{min(hit)}: {s}")
            if s.startswith("scratch_") or re.match(r"buffer_store\w* .*s\[0:3\]", s):
                problems.append(f"{name}: scratch access: {s}")
    return problems


def audit(path):
    with open(path) as fh:
        text = fh.read()
    lines = text.splitlines()
    funcs = split_functions(lines)
    problems = []
    if not funcs:
        problems.append("no conv_wino4w kernels in the assembly")
    for name, body in funcs.items():
        problems += audit_function(name, body)
    # metadata: every conv_wino4w kernel without scratch or spills
    for m in re.finditer(r"\.name:\s+(\S*conv_wino4w\S*)", text):
        pass
    for blk in re.split(r"\n  - ", text.split("amdhsa.kernels:")[-1]):
        nm = re.search(r"\.name:\s+(\S+)", blk)
        if not nm or "conv_wino4w" not in nm.group(1):
            continue
        sp = re.search(r"\.vgpr_spill_count:\s+(\d+)", blk)
        ps = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk)
        if (sp and int(sp.group(1))) or (ps and int(ps.group(1))):
            problems.append(f"{nm.group(1)}: spills / scratch ({sp.group(1) if sp else '?'} VGPR spills, "
                            f"{ps.group(1) if ps else '?'} B private segment)")
    return problems, len(funcs)


def main(argv):
    path = argv[1] if len(argv) > 1 else compile_asm()
    problems, n = audit(path)
    for p in problems:
        print(p)
    print(f"{n} conv_wino4w kernels audited, {len(problems)} findings")
    return 1 if problems else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
