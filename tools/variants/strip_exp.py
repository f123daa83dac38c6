"""Remove the timing-only experiment branches (``MDP_EXP_*``) from C/HIP sources.

The product sources in ``maddpg_amd/csrc`` carry no experiment code; the
experiments live as ``tools/variants/mdp_exp.patch``, which
``tools/build_variant.sh`` applies to a scratch copy before building a
variant with ``-DMDP_EXP_<NAME>``.  This script is how that patch was made
(and how it is regenerated after the product sources change):

    python3 tools/variants/strip_exp.py <dir>        # strip every source in <dir> in place

Every conditional chain whose condition names ``MDP_EXP_`` loses that branch
(the experiment is "not defined" in the product); the chain's remaining
branches are kept, an ``#else`` that becomes the first surviving branch is
emitted unconditionally.  Conditions that mix an experiment macro with other
macros are refused (none exist).
"""
import os
import re
import sys

EXP = "MDP_EXP_"
D_IF = re.compile(r"^\s*#\s*(if|ifdef|ifndef)\b(.*)$")
D_ELIF = re.compile(r"^\s*#\s*elif\b(.*)$")
D_ELSE = re.compile(r"^\s*#\s*else\b")
D_ENDIF = re.compile(r"^\s*#\s*endif\b")


def exp_only(kind, cond):
    """True when the branch is taken only if an experiment macro is defined."""
    c = cond.split("//")[0].strip()
    if EXP not in c:
        return False
    if kind == "ifdef":
        return True
    if kind == "ifndef":
        raise ValueError(f"#ifndef on an experiment macro: {cond!r}")
    # 'defined(MDP_EXP_X)' alone or and-ed with other terms: false whenever X is undefined
    if "||" in c or "!" in c:
        raise ValueError(f"mixed experiment condition: {cond!r}")
    return True


def strip(lines):
    out = []
    # stack entries: None for a chain untouched by experiments, else a dict
    #   emitting: is the current branch emitted; opened: has a surviving #if been written
    stack = []
    for ln in lines:
        m = D_IF.match(ln)
        if m:
            if stack and stack[-1] is not None and not stack[-1]["emitting"]:
                stack.append({"dead": True})        # nested inside a dropped branch
                continue
            if exp_only(m.group(1), m.group(2)):
                stack.append({"emitting": False, "opened": False})
                continue
            stack.append(None)
            out.append(ln)
            continue
        m = D_ELIF.match(ln)
        if m:
            top = stack[-1]
            if top is not None and top.get("dead"):
                continue
            if exp_only("if", m.group(1)):
                if top is None:                       # drop this branch of a product chain
                    stack[-1] = {"emitting": False, "opened": True, "product_chain": True}
                else:
                    top["emitting"] = False
                continue
            if top is None:
                out.append(ln)
            elif top["opened"]:
                top["emitting"] = True
                out.append(ln)
            else:                                     # the first surviving branch opens the chain
                top["emitting"] = top["opened"] = True
                out.append(re.sub(r"#\s*elif", "#if", ln, count=1))
            continue
        if D_ELSE.match(ln):
            top = stack[-1]
            if top is not None and top.get("dead"):
                continue
            if top is None:
                out.append(ln)
            elif top["opened"]:
                top["emitting"] = True
                out.append(ln)
            else:                                     # unconditional from here to #endif
                top["emitting"] = True
                top["bare"] = True
            continue
        if D_ENDIF.match(ln):
            top = stack.pop()
            if top is not None and (top.get("dead") or top.get("bare")):
                continue
            if top is None or top["opened"]:
                out.append(ln)
            continue
        if all(t is None or (not t.get("dead") and t["emitting"]) for t in stack):
            out.append(ln)
    assert not stack, "unbalanced conditionals"
    return out


def main(d):
    for f in sorted(os.listdir(d)):
        if not f.endswith((".hip", ".h", ".cpp")):
            continue
        p = os.path.join(d, f)
        src = open(p).read().splitlines(keepends=True)
        new = strip(src)
        if new != src:
            open(p, "w").write("".join(new))
            print(f"stripped {f}: {len(src) - len(new)} lines")


if __name__ == "__main__":
    main(sys.argv[1])
