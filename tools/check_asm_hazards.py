"""ISA-level check of k_conv4_max's inline-asm screening keys (VERDICT r05 weak
#11): the keys are built by inline asm (screen_key_asm, csrc/feat_fused.hip)
that READS MFMA accumulators, and hipcc pads nothing inside an asm string, so
the MFMA -> VALU-read wait states (12 for an 8-pass XDL op such as
v_mfma_f32_32x32x16_bf16 on gfx950, cdna_hip_programming.md §5.7 item 2)
must come from the instructions the schedule happens to place between the
accumulator's last MFMA and the asm.  This compiles feat_fused.hip for gfx950
(device-only assembly, the Makefile's flags) and, for every asm statement of
every k_conv4_max instantiation, finds the MFMA that last wrote each VGPR the
statement reads - scanning backwards in program order and, past the loop
header, around the loop's back edge - and counts the wait states in between
(one per instruction, N + 1 per s_nop N).  Exit status 1 if any is below the
requirement.

    python tools/check_asm_hazards.py [--need 12] [--asm existing.s]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "adversarial_learning_on_pointclouds_amd", "csrc", "feat_fused.hip")


def compile_asm(out):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17",
           "-I" + os.path.join(REPO, "include"), "--cuda-device-only", "-S", SRC, "-o", out]
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)


REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def functions(lines):
    """{name: [(kind, text)]} for the k_conv4_max kernels; kind in
    'inst', 'label', 'asm' (one asm statement's instructions joined)."""
    funcs, cur, name, in_asm, asm = {}, None, None, False, []
    for ln in lines:
        s = ln.strip()
        m = re.match(r"^(_ZN5pcadv11k_conv4_max\w+):", s)
        if m:
            name, cur = m.group(1), []
            funcs[name] = cur
            continue
        if cur is None:
            continue
        if s.startswith(".Lfunc_end"):
            cur, name = None, None
            continue
        if s.startswith(";;#ASMSTART"):
            in_asm, asm = True, []
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            if asm:
                cur.append(("asm", "\n".join(asm)))
            continue
        if not s or s.startswith(";") or s.startswith("."):
            if re.match(r"^\.LBB\w+:", s):
                cur.append(("label", s[:-1]))
            continue
        if in_asm:
            asm.append(s.split(";")[0].strip())
        else:
            cur.append(("inst", s.split(";")[0].strip()))
    return funcs


def cost(kind, text):
    if kind == "label":
        return 0
    if kind == "asm":
        return sum(cost("inst", t) for t in text.split("\n"))
    m = re.match(r"s_nop\s+(\d+)", text)
    return int(m.group(1)) + 1 if m else 1


def mfma_dst(text):
    if not text.startswith("v_mfma"):
        return set()
    return regs(text.split(",")[0].split(None, 1)[1])


def branch_targets(body):
    """label -> indices of the branches jumping to it."""
    t = {}
    for i, (k, x) in enumerate(body):
        m = re.match(r"s_(?:c)?branch\w*\s+(\.LBB\w+)", x) if k == "inst" else None
        if m:
            t.setdefault(m.group(1), []).append(i)
    return t


def distance(body, i, reg, targets, depth=0):
    """Wait states from the last MFMA writing `reg` before body[i] to body[i]
    along every path backwards (the minimum), None if none within the
    function.  A label reached backwards continues at the instruction before
    it (fall-through) and at every branch that jumps to it (loop back edges)."""
    best = None
    acc = 0
    j = i - 1
    while j >= 0:
        k, x = body[j]
        if k == "inst" and reg in mfma_dst(x):
            return acc if best is None else min(best, acc)
        if k == "label" and depth < 3:
            for b in targets.get(x, []):
                if b >= i:  # a back edge: the path comes from the loop's end
                    d = distance(body, b + 1, reg, targets, depth + 1)
                    if d is not None:
                        best = acc + d if best is None else min(best, acc + d)
        acc += cost(k, x)
        if best is not None and acc >= best:
            return best
        j -= 1
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--need", type=int, default=12)
    ap.add_argument("--asm", default=None, help="an existing assembly listing instead of compiling")
    a = ap.parse_args()
    path = a.asm
    if path is None:
        path = os.path.join(tempfile.mkdtemp(), "feat_fused.s")
        compile_asm(path)
    funcs = functions(open(path).read().splitlines())
    worst, bad, n = None, 0, 0
    for name, body in sorted(funcs.items()):
        targets = branch_targets(body)
        fmin = None
        for i, (k, x) in enumerate(body):
            if k != "asm" or "v_bitop3" not in x and "v_ashrrev" not in x:
                continue
            first = x.split("\n")[0]
            srcs = regs(first.split(",", 1)[1]) if "," in first else set()
            for r in srcs:
                d = distance(body, i, r, targets)
                if d is None:
                    continue
                n += 1
                fmin = d if fmin is None else min(fmin, d)
                if d < a.need:
                    bad += 1
                    print(f"{name}: asm reading v{r} {d} wait states after its MFMA: {first}")
        print(f"{name}: {n} accumulator reads checked so far, minimum distance "
              f"{fmin if fmin is not None else '-'} wait states (need {a.need})")
        if fmin is not None:
            worst = fmin if worst is None else min(worst, fmin)
    print(f"TOTAL reads {n}, minimum {worst}, below {a.need}: {bad}")
    return 1 if bad or n == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
