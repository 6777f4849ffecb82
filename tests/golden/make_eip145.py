"""Generate tests/golden/eip145.json: the EIP-145 SHL/SHR/SAR known answers the reference tests hold
(tests/instructions/shl_test.py:53-125, shr_test.py:56-127, sar_test.py:54-151).

Run in the build container:  python tests/golden/make_eip145.py /root/reference/tests/instructions
Only the (value, shift, expected) hex-string triples are extracted (via ast, as data).
"""
import ast
import json
import sys
from pathlib import Path


def triples(path: Path):
    tree = ast.parse(path.read_text())
    out = []
    for node in ast.walk(tree):
        if isinstance(node, ast.Tuple) and len(node.elts) == 3 and all(
            isinstance(e, ast.Constant) and isinstance(e.value, str) and e.value.startswith("0x")
            for e in node.elts
        ):
            out.append([e.value for e in node.elts])
    return out


def main(root: str) -> None:
    res = {}
    for op in ("shl", "shr", "sar"):
        res[op] = [{"value": v, "shift": s, "expected": e}
                   for v, s, e in triples(Path(root) / ("%s_test.py" % op))]
    dst = Path(__file__).parent / "eip145.json"
    dst.write_text(json.dumps(res, indent=1))
    print({k: len(v) for k, v in res.items()})


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/tests/instructions")
