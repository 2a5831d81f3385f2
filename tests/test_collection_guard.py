"""Guard: no test module defines the same top-level test twice.  Python keeps only
the last definition, so a shadowed test silently stops running (round 3 lost
test_gpu_codec.py's range entry-point cases that way)."""
import ast
import glob
import os

TESTS = os.path.dirname(os.path.abspath(__file__))


def test_no_duplicate_test_names():
    dups = []
    for path in sorted(glob.glob(os.path.join(TESTS, "*.py"))):
        tree = ast.parse(open(path).read(), path)
        seen = {}
        for node in tree.body:
            if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)) and \
                    node.name.startswith(("test_", "Test")):
                if node.name in seen:
                    dups.append(f"{os.path.basename(path)}:{node.lineno} {node.name} "
                                f"(first at line {seen[node.name]})")
                seen.setdefault(node.name, node.lineno)
    assert not dups, dups
