#!/usr/bin/env python3
"""Critical-path / issue bound of a kernel's substep loop from its gfx950 ISA.

    python scripts/critical_path.py build_variants/pob_kernels-hip-amdgcn-amd-amdhsa-gfx950.s \
        k_step_hexILi0EfLb1E [--loop N]

(the .s comes from `hipcc --save-temps` of pob_kernels.hip with the product flags; the kernel
argument is a substring of its mangled name).

What it computes, for the instructions of the chosen loop's body (one iteration = one plain +
one collide substep), taken in layout order along the COMMON path: every block of the loop
except the bodies of inner loops (the per-lane wall / face walks, taken as zero-trip: a wave
with no wall near any of its envs), blocks that call out-of-line functions (the IEEE slow
paths of the range guards) and nothing else skipped -- so every contact branch (ground
contacts, limits, friction) counts as executed, as it is for at least one lane of nearly every
wave:

  issue    sum of the single-wave issue costs (MI355X_MICROARCH.md "vector-instruction ISSUE
           cost, one wave's stream": VALU 4 cycles, transcendental 8, s_nop 4, ...)
  chain    the longest dependency chain through the body's registers with per-class result
           latencies (dependent VALU -> VALU 6 cycles, measured on this repo's microbenchmark,
           DESIGN.md §4; ds_read 50; scalar load 60), issue width unlimited
  inorder  a one-wave in-order timeline: each instruction issues after the previous one's issue
           cost AND after its operands are ready -- the time one wave alone needs for the path
           (what bounds a launch whose waves each have a SIMD to themselves)

All three are cycles per loop iteration; x (substeps / 2) iterations give the physics phase of
one env-step, to be compared with the measured per-wave physics time (phase clocks).
"""
from __future__ import annotations

import argparse
import re
import sys
from collections import defaultdict

TRANS = ("v_rcp_", "v_rsq_", "v_sqrt_", "v_exp_", "v_log_", "v_sin_", "v_cos_", "v_rcp_iflag")
REG_RE = re.compile(r"\b(v|s|a)\[(\d+):(\d+)\]|\b(v|s|a)(\d+)\b|\b(vcc|vcc_lo|vcc_hi|exec|exec_lo|exec_hi|m0|scc)\b")

# single-wave issue cost and result latency (cycles) per class
COST = {"valu": (4, 6), "trans": (8, 10), "v2s": (4, 8), "salu": (2, 2), "smem": (2, 60), "lds_r": (4, 50),
        "lds_w": (4, 0), "vmem_r": (4, 500), "vmem_w": (4, 0), "branch": (8, 0), "nop": (4, 0), "wait": (0, 0),
        "other": (2, 2)}


def classify(m: str) -> str:
    if m.startswith("s_nop"):
        return "nop"
    if m.startswith("s_waitcnt") or m in ("s_setprio", "s_sleep") or m.startswith("s_barrier"):
        return "wait"
    if m.startswith("s_cbranch") or m == "s_branch":
        return "branch"
    if m.startswith("s_load") or m.startswith("s_buffer_load"):
        return "smem"
    if m.startswith("s_"):
        return "salu"
    if m.startswith("ds_read") or m.startswith("ds_load") or m.startswith("ds_bpermute") or m.startswith("ds_swizzle"):
        return "lds_r"
    if m.startswith("ds_"):
        return "lds_w"
    if m.startswith(("global_load", "buffer_load", "flat_load", "scratch_load")):
        return "vmem_r"
    if m.startswith(("global_store", "buffer_store", "flat_store", "scratch_store", "global_atomic")):
        return "vmem_w"
    if m.startswith(("v_readfirstlane", "v_readlane", "v_cmp")):
        return "v2s"
    if m.startswith(TRANS):
        return "trans"
    if m.startswith("v_"):
        return "valu"
    return "other"


def regs(text: str):
    out = []
    for m in REG_RE.finditer(text):
        if m.group(1):
            k, a, b = m.group(1), int(m.group(2)), int(m.group(3))
            out += [f"{k}{i}" for i in range(a, b + 1)]
        elif m.group(4):
            out.append(f"{m.group(4)}{m.group(5)}")
        else:
            n = m.group(6)
            out += {"vcc": ["vcc_lo", "vcc_hi"], "exec": ["exec_lo", "exec_hi"]}.get(n, [n])
    return out


def parse_instr(line: str):
    s = line.split(";")[0].strip()
    if not s or s.endswith(":") or s.startswith("."):
        return None
    parts = s.split(None, 1)
    m = parts[0]
    ops = parts[1] if len(parts) > 1 else ""
    cls = classify(m)
    # split operands at top-level commas; modifiers (dpp, offset:...) follow the last operand
    toks = [t.strip() for t in ops.split(",")] if ops else []
    defs, uses = [], []
    no_def = cls in ("lds_w", "vmem_w", "branch", "nop", "wait") or m.startswith(("s_cmp", "s_bitcmp"))
    if toks and not no_def:
        defs = regs(toks[0])
        uses = regs(",".join(toks[1:]))
    else:
        uses = regs(ops)
    if m.startswith(("s_cmp", "s_bitcmp")) or (m.startswith("s_") and cls == "salu" and not m.startswith("s_mov")):
        defs = defs + ["scc"]
    if m.startswith("s_cbranch_scc") or m.startswith("s_cselect") or m.startswith(("s_addc", "s_subb")):
        uses = uses + ["scc"]
    if m.startswith("s_cbranch_vcc"):
        uses = uses + ["vcc_lo", "vcc_hi"]
    if m.endswith("_e32") and (m.startswith("v_cndmask") or m.startswith(("v_addc", "v_subb"))):
        uses = uses + ["vcc_lo", "vcc_hi"]
    if m.startswith("v_cmpx"):
        defs = defs + ["exec_lo", "exec_hi"]
    return {"m": m, "cls": cls, "defs": defs, "uses": uses, "text": s}


def load_function(path: str, name: str):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + re.escape(name) + r"\w*:", l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, order, cur = {}, [], "__entry"
    blocks[cur] = []
    order.append(cur)
    for l in lines[start + 1:end]:
        lab = re.match(r"^(\.LBB\d+_\d+):", l)
        if lab:
            cur = lab.group(1)
            blocks[cur] = []
            order.append(cur)
            continue
        ins = parse_instr(l)
        if ins:
            blocks[cur].append(ins)
    return blocks, order


def cfg(blocks, order):
    """successors of every block (fall-through and branch targets)"""
    succ = {}
    for i, b in enumerate(order):
        bl = blocks[b]
        nxt = order[i + 1] if i + 1 < len(order) else None
        out = []
        last = bl[-1] if bl else None
        if last is not None and last["cls"] == "branch":
            out.append(last["text"].split()[-1])
            if last["m"] != "s_branch" and nxt:
                out.append(nxt)
        elif last is not None and (last["m"] == "s_endpgm" or last["m"].startswith("s_setpc")):
            pass
        elif nxt:
            out.append(nxt)
        succ[b] = [x for x in out if x in blocks]
    return succ


def natural_loops(blocks, order, succ):
    """(header, set of blocks) of every natural loop, from the DFS back edges"""
    pred = defaultdict(list)
    for b, ss in succ.items():
        for x in ss:
            pred[x].append(b)
    state, back = {}, []
    stack = [(order[0], iter(succ[order[0]]))]
    state[order[0]] = 1
    while stack:
        b, it = stack[-1]
        nxt = next(it, None)
        if nxt is None:
            state[b] = 2
            stack.pop()
            continue
        if state.get(nxt) == 1:
            back.append((b, nxt))
        elif nxt not in state:
            state[nxt] = 1
            stack.append((nxt, iter(succ[nxt])))
    loops = defaultdict(set)
    for u, h in back:
        body = {h, u}
        work = [u]
        while work:
            x = work.pop()
            if x == h:
                continue
            for p in pred[x]:
                if p not in body:
                    body.add(p)
                    work.append(p)
        loops[h] |= body
    return dict(loops)


def rpo(blocks, succ, entry, allowed):
    seen, out = set(), []
    stack = [(entry, iter([x for x in succ[entry] if x in allowed]))]
    seen.add(entry)
    while stack:
        b, it = stack[-1]
        nxt = next(it, None)
        if nxt is None:
            out.append(b)
            stack.pop()
            continue
        if nxt not in seen:
            seen.add(nxt)
            stack.append((nxt, iter([x for x in succ[nxt] if x in allowed])))
    return out[::-1]


def analyse(blocks, order, succ, hdr, body, all_loops):
    inner = [(h, bd) for h, bd in all_loops.items() if h != hdr and h in body and bd < body]
    skip = set()
    for h, bd in inner:
        skip |= bd
    calls = {b for b in body if any(i["m"].startswith(("s_swappc", "s_setpc")) for i in blocks[b])}
    allowed = (body - skip - calls)
    # inner loops run zero trips: an edge into one continues at its exits; a call block is
    # passed through to its successors (the slow path not taken)
    outer_inner = [bd for h, bd in inner if not any(bd < bd2 for _, bd2 in inner)]

    def redirect(x, seen=None):
        seen = seen or set()
        if x in seen:
            return []
        seen.add(x)
        for bd in outer_inner:
            if x in bd:
                exits = {y for b in bd for y in succ[b] if y not in bd}
                return [z for y in exits for z in redirect(y, seen)]
        if x in calls:
            return [z for y in succ[x] for z in redirect(y, seen)]
        return [x]
    fsucc = {b: sorted({z for x in succ[b] if x != hdr for z in redirect(x)}, key=order.index) for b in succ}
    # execution order: reverse post-order from the header over the loop's forward edges
    seq = rpo(blocks, fsucc, hdr, allowed)
    path = [ins for b in seq for ins in blocks[b]]
    issue = sum(COST[ins["cls"]][0] for ins in path)
    ready = defaultdict(float)
    chain_ready = defaultdict(float)
    t = 0.0
    chain = 0.0
    counts = defaultdict(int)
    for ins in path:
        iss, lat = COST[ins["cls"]]
        counts[ins["cls"]] += 1
        dep = max((ready[r] for r in ins["uses"]), default=0.0)
        start = max(t, dep)
        for r in ins["defs"]:
            ready[r] = start + max(lat, 1)
        t = start + iss
        cdep = max((chain_ready[r] for r in ins["uses"]), default=0.0)
        for r in ins["defs"]:
            chain_ready[r] = cdep + max(lat, 1)
        chain = max(chain, cdep + lat)
    return {"instructions": len(path), "blocks": len(seq), "by_class": dict(counts), "issue": issue, "chain": chain,
            "inorder": t, "inner_loops_skipped": len(inner), "call_blocks_skipped": len(calls & body)}


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--loop", type=int, default=-1, help="index of the outer loop (default: the largest)")
    ap.add_argument("--iters", type=int, default=5, help="loop iterations per env-step (substeps / 2)")
    ap.add_argument("--ghz", type=float, default=2.4)
    ap.add_argument("--inner", action="store_true",
                    help="also analyse each inner loop of the chosen loop (one trip of its body: the wall "
                         "walks' cost per face item), every block of it counted as executed")
    a = ap.parse_args()
    blocks, order = load_function(a.asm, a.kernel)
    succ = cfg(blocks, order)
    L = natural_loops(blocks, order, succ)
    # outer loops: not contained in another loop
    outer = [(h, bd) for h, bd in L.items() if not any(h2 != h and bd < bd2 for h2, bd2 in L.items())]
    size = lambda bd: sum(len(blocks[b]) for b in bd)  # noqa: E731
    outer.sort(key=lambda x: size(x[1]), reverse=True)
    for k, (h, bd) in enumerate(outer[:4]):
        print(f"outer loop {k}: header {h}, {len(bd)} blocks, {size(bd)} instructions")
    h, bd = outer[a.loop] if a.loop >= 0 else outer[0]
    r = analyse(blocks, order, succ, h, bd, L)
    print(f"kernel {a.kernel}, loop {h}: {r['instructions']} instructions in {r['blocks']} blocks on the common path "
          f"({r['inner_loops_skipped']} inner loops as zero-trip, {r['call_blocks_skipped']} call blocks skipped)")
    print(f"  by class: {r['by_class']}")
    if a.inner:
        for hi, bdi in sorted(((x, y) for x, y in L.items() if x != h and x in bd and y < bd), key=lambda z: order.index(z[0])):
            ri = analyse(blocks, order, succ, hi, bdi, L)
            print(f"  inner loop {hi}: {len(bdi)} blocks, {size(bdi)} instructions; one trip: {ri['instructions']} "
                  f"instructions, issue {ri['issue']:.0f} / chain {ri['chain']:.0f} / inorder {ri['inorder']:.0f} cycles, "
                  f"{ri['by_class'].get('valu', 0)} VALU")
    us = lambda c: c * a.iters / (a.ghz * 1e3)  # noqa: E731
    for k in ("issue", "chain", "inorder"):
        print(f"  {k:8s} {r[k]:9.0f} cycles / iteration  -> x{a.iters} = {r[k] * a.iters:9.0f} cycles "
              f"= {us(r[k]):6.2f} us at {a.ghz} GHz")


if __name__ == "__main__":
    main()
