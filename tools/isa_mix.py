"""Static VALU mix of a kernel in gfx950 assembly, split at s_memtime marks
(the phase-profiling build) or whole: counts per segment of full-rate and
half-rate VALU opcodes (profiles/r02_valu_ops.txt), SGPR-operand VALU (half
rate whatever the opcode), LDS and VMEM instructions.  Static counts: a loop
body counts once.
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -S \\
          [-DORBX_PHASE_PROF] -o /tmp/x.s orb_slam_2_ros_amd/csrc/orbx_extract.hip
    python tools/isa_mix.py /tmp/x.s k_fastILb0 [--ops]"""
import re
import sys
from collections import Counter

FULL = {"v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_lshrrev_b32",
        "v_min_u16", "v_max_u16", "v_sub_u16", "v_add_u16", "v_min_i16", "v_max_i16", "v_add_f32", "v_sub_f32",
        "v_subrev_f32", "v_mul_f32", "v_fmac_f32", "v_fma_f32", "v_mov_b32", "v_not_b32", "v_mac_f32"}
SGPR = re.compile(r"(?<![a-z_])(s\d+|s\[\d+:\d+\]|vcc|vcc_lo|vcc_hi|exec|ttmp\d+)(?![\w:])")


def main():
    path, fn = sys.argv[1], sys.argv[2]
    show_ops = "--ops" in sys.argv
    lines = open(path).read().splitlines()
    start = next(i for i, ln in enumerate(lines) if re.match(r"^_Z\w*" + re.escape(fn) + r"\w*:", ln))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    segs = [Counter()]
    ops = [Counter()]
    for ln in lines[start:end]:
        t = ln.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if op == "s_memtime":
            segs.append(Counter())
            ops.append(Counter())
            continue
        c = segs[-1]
        if op.startswith("v_"):
            base = re.sub(r"_e(32|64)$|_dpp$|_sdwa$", "", op)
            args = t[len(op):]
            if "_dpp" in op or "row_" in args or "quad_perm" in args:
                c["half"] += 1
            elif base in FULL and not SGPR.search(args.split(";")[0]):
                c["full"] += 1
            else:
                c["half"] += 1
                if base in FULL:
                    c["full_op_sgpr"] += 1
            ops[-1][base] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            c["vmem"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    tot = sum(segs, Counter())
    print(f"total: full {tot['full']}  half {tot['half']}  half-rate equivalents {tot['half'] + tot['full'] / 2:.1f}  "
          f"pk_f32 {sum(o[k] for o in ops for k in o if k.startswith('v_pk_') and k.endswith('_f32'))}")
    for i, c in enumerate(segs):
        eq = c["half"] + c["full"] / 2
        print(f"segment {i}: full {c['full']:4d}  half {c['half']:4d} (of which full-rate opcode with an SGPR "
              f"operand {c['full_op_sgpr']:3d})  half-rate equivalents {eq:6.1f}  lds {c['lds']:3d}  vmem {c['vmem']:3d}"
              f"  salu {c['salu']:4d}")
        if show_ops:
            print("   ", ", ".join(f"{k} {v}" for k, v in ops[i].most_common(25)))


if __name__ == "__main__":
    main()
