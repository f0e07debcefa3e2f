"""Lane-stack budget of the recursive evaluator, from the product ISA.

The evaluator recurses (eval_conj <-> clauses, query filters, rule references, count()) in a dynamic lane
stack of 16 KB (capi.cpp).  It reads its stack pointer where it recurses (eval_core.inc stack_low, marked
`gg_stack_check` in the assembly) and ends the tile with E_STACK past `stack limit - kStackMargin`.  This
tool reads every function's own frame and its callees from the assembly's `.private_seg_size` expressions
and computes the largest stack growth from a passing check to the next check (or to the deepest leaf):
the margin must cover it.

  hipcc --offload-arch=gfx950 <eval_kernel.o's flags> --cuda-device-only -S csrc/eval_kernel.hip -o k.s
  python tools/stack_budget.py k.s [margin]
"""
import re
import sys
from collections import defaultdict

# functions whose stack check runs before any call they make (the check is the first thing the clause
# dispatcher / query driver / function resolver does)
CHECKED = ("9eval_conj", "15query_retrieval", "16resolve_function")
# resolve_let: its inlined query driver checks before walking, but its count() branch calls
# resolve_function (itself checked) first
PARTIAL = ("11resolve_let",)


def parse(path):
    own, callees, marked = {}, defaultdict(list), set()
    cur = None
    for line in open(path):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
        if "gg_stack_check" in line and cur:
            marked.add(cur)
        # calls: the callee's address is formed from its symbol (`s_add_u32 sN, sN, <callee>@rel32@lo+4`);
        # the .private_seg_size expressions omit callees inside a recursive cycle, so edges come from here
        m = re.search(r"(_Z\S+)@rel32@lo", line)
        if m and cur and m.group(1) not in callees[cur]:
            callees[cur].append(m.group(1))
        m = re.match(r"\s*\.set (\S+)\.private_seg_size, (.*)$", line)
        if m:
            name, expr = m.group(1).lstrip("."), m.group(2)
            name = name[1:] if name.startswith("L_") else name
            n = re.match(r"(\d+)", expr)
            own[name] = int(n.group(1)) if n else 0
    return own, callees, marked


def budget(path):
    own, callees, marked = parse(path)
    checked = {f for f in own if any(k in f for k in CHECKED)}
    partial = {f for f in own if any(k in f for k in PARTIAL)}
    memo = {}

    def chain(f, stack=()):
        # growth from entering f to f's first check (checked functions) or to its deepest leaf
        if f in checked:
            return own[f]
        if f in memo:
            return memo[f]
        if f in stack:
            raise SystemExit("unchecked recursion through %s" % " -> ".join(stack + (f,)))
        if f in partial:   # its own check covers every callee but resolve_function
            sub = [chain(g, stack + (f,)) for g in callees[f] if "16resolve_function" in g]
        else:
            sub = [chain(g, stack + (f,)) for g in callees[f] if g in own]
        memo[f] = own[f] + max(sub or [0])
        return memo[f]

    worst = []
    for f in sorted(checked | partial):
        after = max([chain(g) for g in callees[f] if g in own] or [0])
        worst.append((after, f))
    worst.sort(reverse=True)
    return worst, checked, marked


if __name__ == "__main__":
    worst, checked, marked = budget(sys.argv[1])
    margin = int(sys.argv[2]) if len(sys.argv) > 2 else 3072
    missing = sorted(f for f in checked if f not in marked)
    for after, f in worst[:8]:
        print("%6d B after the check in %s" % (after, f))
    if missing:
        print("functions treated as checked but without a gg_stack_check:", missing)
    x = worst[0][0] if worst else 0
    print("largest growth between checks: %d B; kStackMargin %d B: %s" % (x, margin, "ok" if x < margin and not missing else "TOO SMALL"))
    sys.exit(0 if x < margin and not missing else 1)
