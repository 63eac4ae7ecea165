"""Reference-semantics oracles without importing the (broken, F8) reference modules.

Functions/classes are extracted from /root/reference with ``ast`` and executed in a
namespace we control.  Tests using this skip when the reference tree is
absent (e.g. on the GPU box, which only receives /root/repo).
"""
import ast
import os

import pytest

REF = '/root/reference'
needs_ref = pytest.mark.skipif(not os.path.isdir(REF), reason='reference tree not mounted')


def extract(relpath, names, namespace):
    src = open(os.path.join(REF, relpath)).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body
            if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.name in names]
    mod = ast.Module(body=keep, type_ignores=[])
    exec(compile(mod, relpath, 'exec'), namespace)
    return namespace


def extract_method(relpath, cls, meth):
    src = open(os.path.join(REF, relpath)).read()
    tree = ast.parse(src)
    for n in tree.body:
        if isinstance(n, ast.ClassDef) and n.name == cls:
            for m in n.body:
                if isinstance(m, ast.FunctionDef) and m.name == meth:
                    return ast.get_source_segment(src, m)
    raise KeyError(meth)
