"""Per-loop instruction mix of a kernel in device assembly (hipcc -S output).

    python tools/asm_loops.py FILE.s KERNEL_SUBSTRING [DEPTH]

The compiler annotates every basic block of a loop with "in Loop: Header=BBx_y Depth=d" (the
header block: "Loop Header: Depth=d"). For each loop this prints the instruction counts of the
blocks that belong to it (nested loops included): VALU (FP64), LDS, SALU, scratch, calls, so the
record loop of k_modesum (the one holding the fast path's v_rsq_f64) can be told apart from the
list build and the cold pass.
"""
import re
import sys


def blocks(body):
    """[(label, header_of_innermost_loop_or_None, depth, lines)]"""
    out, cur = [], None
    for l in body:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):(.*)$", l)
        if m:
            cur = [m.group(1), None, 0, []]
            out.append(cur)
            ann = m.group(2)
        elif cur is None:
            continue
        else:
            ann = l if l.strip().startswith(";") and "Loop" in l else ""
        a = re.search(r"Header=BB(\d+_\d+) Depth=(\d+)", ann)
        if a:
            cur[1], cur[2] = ".LBB" + a.group(1), int(a.group(2))
        elif re.search(r"Loop Header: Depth=(\d+)", ann):
            cur[1] = cur[0] if cur[0].startswith(".LBB") else cur[1]
            cur[2] = int(re.search(r"Depth=(\d+)", ann).group(1))
        if not m:
            cur[3].append(l)
    return out


def main(path, kname, want_depth=None):
    L = open(path).read().split("\n")
    s = next(i for i, l in enumerate(L) if l.startswith("_ZN") and kname in l and ":" in l)
    e = next(i for i in range(s, len(L)) if L[i].startswith(".Lfunc_end"))
    bl = blocks(L[s:e])
    parent = {}
    for lab, hdr, d, _ in bl:
        if hdr and hdr == lab:
            pass
    heads = {}
    for lab, hdr, d, _ in bl:
        if hdr:
            heads.setdefault(hdr, d)
    # a block belongs to loop H if its innermost header is H or a loop nested in H; nesting from
    # block order: a header of depth d+1 inside H's span
    order = [b[0] for b in bl]
    for H, d in sorted(heads.items(), key=lambda x: order.index(x[0]) if x[0] in order else 0):
        if want_depth is not None and d != want_depth:
            continue
        idx = [i for i, b in enumerate(bl) if b[1] == H]
        lo, hi = min(idx), max(idx)
        ins = [x.strip().split()[0] for b in bl[lo:hi + 1] for x in b[3]
               if x.strip() and not x.strip().startswith((";", "."))]
        v = [i for i in ins if i.startswith("v_")]
        print(f"{H} depth {d} blocks {lo}-{hi}: valu {len(v)} (f64 {sum('f64' in i for i in v)}) "
              f"ds {sum(i.startswith('ds_') for i in ins)} salu {sum(i.startswith('s_') for i in ins)} "
              f"scratch {sum('scratch' in i for i in ins)} calls {sum('swappc' in i for i in ins)} "
              f"rsq {sum('v_rsq_f64' in i for i in ins)}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else None)
