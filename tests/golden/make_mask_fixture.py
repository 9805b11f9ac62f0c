"""Extract the index sets of po_brax/standard_observability_masks.py:5-67 as DATA.

Run once in the build container (the reference is not on the GPU box):
    python tests/golden/make_mask_fixture.py /root/reference/po_brax/standard_observability_masks.py
The reference module imports brax (absent here), so it is not imported: its source is
parsed with ``ast`` and the ``jp.arange(a, b)`` / ``jp.concatenate((...), axis=0)`` calls of
each dict entry are expanded to explicit index lists, written to
tests/golden/observability_masks.json (dict name -> env name -> [indices]).
"""
import ast
import json
import os
import sys


def _expand(node):
    if isinstance(node, ast.Call):
        fn = node.func.attr if isinstance(node.func, ast.Attribute) else node.func.id
        if fn == "arange":
            a, b = (ast.literal_eval(x) for x in node.args)
            return list(range(a, b))
        if fn == "concatenate":
            out = []
            for part in node.args[0].elts:
                out += _expand(part)
            return out
    raise ValueError(f"unexpected expression {ast.dump(node)}")


def main(src, dst):
    tree = ast.parse(open(src).read())
    out = {}
    for stmt in tree.body:
        if isinstance(stmt, ast.Assign) and isinstance(stmt.value, ast.Dict):
            name = stmt.targets[0].id
            out[name] = {ast.literal_eval(k): _expand(v) for k, v in zip(stmt.value.keys, stmt.value.values)}
    json.dump({"source": "po_brax/standard_observability_masks.py:5-67 (parsed, not imported)", "masks": out},
              open(dst, "w"), indent=None, separators=(",", ":"))
    print({k: len(v) for k, v in out.items()})


if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/po_brax/standard_observability_masks.py",
         os.path.join(here, "observability_masks.json"))
