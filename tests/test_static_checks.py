"""CPU-side static checks of the native op layer (GPU-only code paths cannot run here)."""
import ast
import glob
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _count(v):
    if isinstance(v, ast.Tuple):
        return len(v.elts)
    if isinstance(v, ast.BinOp) and isinstance(v.op, ast.Mult) and isinstance(v.left, ast.Tuple) \
            and isinstance(v.right, ast.Constant):
        return len(v.left.elts) * v.right.value
    if isinstance(v, ast.BinOp) and isinstance(v.op, ast.Add):
        a, b = _count(v.left), _count(v.right)
        return None if a is None or b is None else a + b
    return None


def test_autograd_functions_return_one_gradient_per_input():
    """Every autograd.Function backward in deep_vision_amd/ returns exactly as many gradients as
    its forward takes inputs (a mismatch only surfaces on the GPU otherwise)."""
    bad = []
    for f in glob.glob(os.path.join(ROOT, "deep_vision_amd", "**", "*.py"), recursive=True):
        tree = ast.parse(open(f).read())
        for c in [n for n in ast.walk(tree) if isinstance(n, ast.ClassDef)]:
            fw = [n for n in c.body if isinstance(n, ast.FunctionDef) and n.name == "forward"]
            bw = [n for n in c.body if isinstance(n, ast.FunctionDef) and n.name == "backward"]
            if not fw or not bw or fw[0].args.vararg:
                continue
            nin = len(fw[0].args.args) - 1  # minus ctx
            for r in ast.walk(bw[0]):
                if isinstance(r, ast.Return) and r.value is not None:
                    n = _count(r.value)
                    if n is not None and n != nin and nin > 1:
                        bad.append(f"{os.path.relpath(f, ROOT)}:{r.lineno} {c.name} returns {n}, forward takes {nin}")
    assert not bad, "\n".join(bad)
