"""Dygraph-to-static control-flow conversion (parity: python/paddle/jit/dy2static/
convert_operators.py ``convert_ifelse`` :315 / ``convert_while_loop`` :94 /
``convert_logical_and|or|not``, produced by ifelse_transformer.py, loop_transformer.py and
return_transformer.py).

``convert_function(fn)`` rewrites the source of ``fn`` so that every ``if`` / ``while`` whose
test may be a tensor becomes a call into this module:

    if <test>:                         def __pra_true_0(__pra_v):
        <body>                             (a, b) = __pra_v
    else:                 ==>              <body>; return (a, b)
        <orelse>                       def __pra_false_0(__pra_v): ...
                                       (a, b) = _jst.convert_ifelse(<test>, __pra_true_0,
                                                                    __pra_false_0, _jst.pack(...))

(``a``, ``b`` = every name either branch assigns), and ``while`` likewise into
``convert_while_loop(cond_fn, body_fn, vals)``. At run time the converters look at the test's
value: a Python bool or an eager tensor takes the Python branch / loop (eager semantics are
unchanged), a static ``Variable`` (program recording for ``jit.save`` / ``concrete_program``)
builds ``static.nn.cond`` / ``static.nn.while_loop`` sub-blocks, so the saved program holds
BOTH branches and the loop, decided by the fed values when it runs. ``and`` / ``or`` / ``not``
in tests become ``convert_logical_*``. Early returns (``if c: return x`` followed by more
code) are first folded into an ``else`` so both branches end in a return.

Not converted (left as Python): loops with ``break`` / ``continue`` / ``return`` inside,
``for`` loops, branches that return in the middle.
"""
import ast
import functools
import inspect
import textwrap
import types

import torch

__all__ = ['convert_function', 'convert_ifelse', 'convert_while_loop', 'convert_logical_and',
           'convert_logical_or', 'convert_logical_not', 'UNDEFINED']


class _Undefined:
    """A name not bound yet when a converted ``if`` / ``while`` starts."""

    def __repr__(self):
        return 'UNDEFINED'


UNDEFINED = _Undefined()


def pack(env, names):
    return tuple(env.get(n, UNDEFINED) for n in names)


def _is_var(x):
    from ..static import graph as G
    return G._STATIC[0] and isinstance(x, G.Variable)


def _truth(x):
    from ..framework.core import Tensor, _u
    if isinstance(x, Tensor):
        return bool(_u(x).reshape(-1)[0])
    if isinstance(x, torch.Tensor):
        return bool(x.reshape(-1)[0])
    return bool(x)


# -- runtime converters ------------------------------------------------------------------------
def convert_ifelse(pred, true_fn, false_fn, vals):
    if not _is_var(pred):
        return true_fn(vals) if _truth(pred) else false_fn(vals)
    from ..static import graph as G
    from ..static.control_flow import cond
    seen = {}

    def branch(fn, key):
        def run():
            out = fn(vals)
            seen[key] = out
            return [o for o in _flat_out(out) if isinstance(o, G.Variable)]
        return run
    outs = cond(pred, branch(true_fn, 't'), branch(false_fn, 'f'))
    t_out, f_out = seen['t'], seen['f']
    tf, ff = _flat_out(t_out), _flat_out(f_out)
    it = iter(outs if isinstance(outs, (list, tuple)) else [outs])
    merged = []
    for a, b in zip(tf, ff):
        if isinstance(a, G.Variable) != isinstance(b, G.Variable):
            raise ValueError("dy2static: a variable assigned by only one branch of a tensor-valued "
                             "'if' is a tensor in one branch and not in the other")
        if isinstance(a, G.Variable):
            merged.append(next(it))
        elif a is b or _same_const(a, b):
            merged.append(a)
        else:
            raise ValueError(f"dy2static: the branches of a tensor-valued 'if' leave different "
                             f"non-tensor values ({a!r} vs {b!r})")
    return _rebuild_like(t_out, iter(merged))


def _same_const(a, b):
    try:
        return type(a) is type(b) and bool(a == b)
    except Exception:  # noqa: BLE001
        return False


def _flat_out(o):
    if isinstance(o, (list, tuple)):
        r = []
        for x in o:
            r += _flat_out(x)
        return r
    return [o]


def _rebuild_like(tmpl, it):
    if isinstance(tmpl, (list, tuple)):
        return type(tmpl)(_rebuild_like(x, it) for x in tmpl)
    return next(it)


def convert_while_loop(cond_fn, body_fn, vals):
    c = cond_fn(vals)
    if not _is_var(c):
        while _truth(c):
            vals = body_fn(vals)
            c = cond_fn(vals)
        return vals
    from ..framework.core import Tensor
    from ..static.control_flow import while_loop
    # names first bound inside the body are body temporaries, not loop-carried
    keep = [i for i, v in enumerate(vals) if v is not UNDEFINED]
    lv = []
    for i in keep:
        v = vals[i]
        if isinstance(v, (bool, int, float)):
            v = Tensor(torch.tensor(v))
        lv.append(v)

    def full(vs):
        f = list(vals)
        for i, v in zip(keep, vs):
            f[i] = v
        return tuple(f)

    def c2(*vs):
        return cond_fn(full(vs))

    def b2(*vs):
        out = body_fn(full(vs))
        return [out[i] for i in keep]
    res = while_loop(c2, b2, lv)
    return full(res)


def convert_logical_and(*thunks):
    from .. import tensor as T
    v = thunks[0]()
    for th in thunks[1:]:
        if _is_var(v):
            v = T.logical_and(v, th())
        elif not _truth(v):
            return v
        else:
            v = th()
    return v


def convert_logical_or(*thunks):
    from .. import tensor as T
    v = thunks[0]()
    for th in thunks[1:]:
        if _is_var(v):
            v = T.logical_or(v, th())
        elif _truth(v):
            return v
        else:
            v = th()
    return v


def convert_logical_not(x):
    if _is_var(x):
        from .. import tensor as T
        return T.logical_not(x)
    return not _truth(x)


# -- source transformation ---------------------------------------------------------------------
def _stored_names(stmts):
    """Names bound by these statements (not inside nested functions / lambdas / classes)."""
    out = []

    class V(ast.NodeVisitor):
        def visit_Name(self, n):
            if isinstance(n.ctx, ast.Store) and n.id not in out:
                out.append(n.id)

        def visit_FunctionDef(self, n):
            if n.name not in out:
                out.append(n.name)

        visit_AsyncFunctionDef = visit_FunctionDef

        def visit_ClassDef(self, n):
            if n.name not in out:
                out.append(n.name)

        def visit_Lambda(self, n):
            pass

        def visit_ListComp(self, n):
            pass

        visit_SetComp = visit_DictComp = visit_GeneratorExp = visit_ListComp
    v = V()
    for s in stmts:
        v.visit(s)
    return [n for n in out if not n.startswith('__pra_')]


def _contains(stmts, kinds, stop_at_loops=False):
    class V(ast.NodeVisitor):
        found = False

        def generic_visit(self, n):
            if isinstance(n, kinds):
                self.found = True
            if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda, ast.ClassDef)):
                return
            if stop_at_loops and isinstance(n, (ast.For, ast.While)):
                return
            super().generic_visit(n)
    v = V()
    for s in stmts:
        v.generic_visit(s)
        if v.found:
            return True
    return False


def _ends_with_return(stmts):
    return bool(stmts) and isinstance(stmts[-1], ast.Return)


def _fold_early_returns(stmts):
    """``if c: ...; return x`` + rest  ->  ``if c: ...; return x  else: rest`` (recursively)."""
    out = []
    i = 0
    while i < len(stmts):
        s = stmts[i]
        for fld in ('body', 'orelse'):
            if isinstance(s, (ast.If, ast.While, ast.For, ast.With, ast.Try)) and hasattr(s, fld):
                setattr(s, fld, _fold_early_returns(getattr(s, fld)))
        if isinstance(s, ast.If) and i + 1 < len(stmts):
            rest = stmts[i + 1:]
            if _ends_with_return(s.body) and not s.orelse:
                s.orelse = _fold_early_returns(rest)
                out.append(s)
                return out
            if _ends_with_return(s.orelse) and not _contains(s.body, (ast.Return,)):
                s.body = s.body + _fold_early_returns(rest)
                out.append(s)
                return out
        out.append(s)
        i += 1
    return out


class _Transformer(ast.NodeTransformer):
    def __init__(self):
        self.n = 0

    def _uid(self):
        self.n += 1
        return self.n - 1

    def visit_FunctionDef(self, node):
        return node  # nested defs are left alone (only the converted function's own body)

    visit_AsyncFunctionDef = visit_FunctionDef

    def visit_Lambda(self, node):
        return node

    # tests: and / or / not
    def _test(self, e):
        if isinstance(e, ast.BoolOp):
            fn = 'convert_logical_and' if isinstance(e.op, ast.And) else 'convert_logical_or'
            args = [ast.Lambda(args=_no_args(), body=self._test(v)) for v in e.values]
            return _call(fn, args)
        if isinstance(e, ast.UnaryOp) and isinstance(e.op, ast.Not):
            return _call('convert_logical_not', [self._test(e.operand)])
        return e

    def _branch_fn(self, name, names, body, ret_value):
        stmts = []
        if names:
            stmts.append(ast.Assign(targets=[_tuple(names, ast.Store())],
                                    value=ast.Name('__pra_v', ast.Load())))
        stmts += body or [ast.Pass()]
        if ret_value:
            stmts.append(ast.Return(value=_tuple(names, ast.Load())))
        return ast.FunctionDef(name=name, args=_one_arg('__pra_v'), body=stmts, decorator_list=[],
                               returns=None, type_comment=None)

    def visit_If(self, node):
        node = self.generic_visit(node)
        body, orelse = node.body, node.orelse
        returns_both = _ends_with_return(body) and _ends_with_return(orelse)
        inner_ret = _contains(body[:-1] if returns_both else body, (ast.Return,)) or \
            _contains(orelse[:-1] if returns_both else orelse, (ast.Return,))
        if inner_ret or (_contains(body + orelse, (ast.Return,)) and not returns_both):
            return node  # returns we cannot fold: keep Python semantics
        if _contains(body + orelse, (ast.Break, ast.Continue), stop_at_loops=True):
            return node
        k = self._uid()
        names = _stored_names(body + orelse)
        tname, fname = f'__pra_true_{k}', f'__pra_false_{k}'
        if returns_both:
            tf = self._branch_fn(tname, names, body, False)
            ff = self._branch_fn(fname, names, orelse, False)
            call = _call('convert_ifelse', [self._test(node.test), ast.Name(tname, ast.Load()),
                                             ast.Name(fname, ast.Load()), _pack(names)])
            return [tf, ff, ast.Return(value=call)]
        tf = self._branch_fn(tname, names, body, True)
        ff = self._branch_fn(fname, names, orelse, True)
        call = _call('convert_ifelse', [self._test(node.test), ast.Name(tname, ast.Load()),
                                         ast.Name(fname, ast.Load()), _pack(names)])
        if not names:
            return [tf, ff, ast.Expr(value=call)]
        return [tf, ff, ast.Assign(targets=[_tuple(names, ast.Store())], value=call)]

    def visit_While(self, node):
        node = self.generic_visit(node)
        if node.orelse or _contains(node.body, (ast.Break, ast.Continue, ast.Return),
                                    stop_at_loops=True):
            return node
        k = self._uid()
        names = _stored_names(node.body)
        if not names:
            return node
        cname, bname = f'__pra_cond_{k}', f'__pra_body_{k}'
        cfn = ast.FunctionDef(
            name=cname, args=_one_arg('__pra_v'),
            body=[ast.Assign(targets=[_tuple(names, ast.Store())], value=ast.Name('__pra_v', ast.Load())),
                  ast.Return(value=self._test(node.test))],
            decorator_list=[], returns=None, type_comment=None)
        bfn = self._branch_fn(bname, names, node.body, True)
        call = _call('convert_while_loop', [ast.Name(cname, ast.Load()), ast.Name(bname, ast.Load()),
                                             _pack(names)])
        return [cfn, bfn, ast.Assign(targets=[_tuple(names, ast.Store())], value=call)]


def _no_args():
    return ast.arguments(posonlyargs=[], args=[], vararg=None, kwonlyargs=[], kw_defaults=[],
                         kwarg=None, defaults=[])


def _one_arg(name):
    return ast.arguments(posonlyargs=[], args=[ast.arg(arg=name)], vararg=None, kwonlyargs=[],
                         kw_defaults=[], kwarg=None, defaults=[])


def _tuple(names, ctx):
    return ast.Tuple(elts=[ast.Name(n, ctx) for n in names], ctx=ctx)


def _call(fn, args):
    return ast.Call(func=ast.Attribute(value=ast.Name('_pra_jst', ast.Load()), attr=fn,
                                       ctx=ast.Load()), args=args, keywords=[])


def _pack(names):
    return _call('pack', [ast.Call(func=ast.Name('locals', ast.Load()), args=[], keywords=[]),
                          ast.Tuple(elts=[ast.Constant(n) for n in names], ctx=ast.Load())])


def _source_tree(fn):
    src = textwrap.dedent(inspect.getsource(fn))
    tree = ast.parse(src)
    fdef = tree.body[0]
    if not isinstance(fdef, (ast.FunctionDef, ast.AsyncFunctionDef)):
        raise TypeError("dy2static converts functions")
    fdef.decorator_list = []  # no re-entry into to_static
    return tree, fdef


@functools.lru_cache(maxsize=None)
def _convert_code(func):
    """Compile the converted ``func`` inside a factory whose parameters are the original's free
    variables (+ ``_pra_jst``), itself inside a class statement named like the owning class:
    the rebuilt function then has real closure cells (``nonlocal`` writes, zero-argument
    ``super()`` through ``__class__``) and the owner's private-name mangling. Returns the inner
    code object, or None when there is nothing to convert."""
    import sys
    tree, fdef = _source_tree(func)
    fdef.body = _fold_early_returns(fdef.body)
    tr = _Transformer()
    fdef.body = [x for s in fdef.body for x in _as_list(tr.visit(s))]
    if tr.n == 0:
        return None
    params = [n for n in func.__code__.co_freevars if n != '__class__'] + ['_pra_jst']
    factory = ast.FunctionDef(
        name='_pra_factory',
        args=ast.arguments(posonlyargs=[], args=[ast.arg(arg=p) for p in params], vararg=None,
                           kwonlyargs=[], kw_defaults=[], kwarg=None, defaults=[]),
        body=[fdef, ast.Return(value=ast.Name(fdef.name, ast.Load()))], decorator_list=[],
        returns=None, type_comment=None)
    parts = func.__qualname__.split('.')
    owner = parts[-2] if len(parts) >= 2 and parts[-2] != '<locals>' else None
    body = [ast.ClassDef(name=owner, bases=[], keywords=[], body=[factory], decorator_list=[])] \
        if owner else [factory]
    mod = ast.Module(body=body, type_ignores=[])
    ast.fix_missing_locations(mod)
    code = compile(mod, filename=f'<dy2static {func.__qualname__}>', mode='exec')

    def find(c, name):
        for k in c.co_consts:
            if isinstance(k, types.CodeType):
                if k.co_name == name:
                    return k
                r = find(k, name)
                if r is not None:
                    return r
        return None
    fac = find(code, '_pra_factory')
    inner = next(k for k in fac.co_consts if isinstance(k, types.CodeType) and k.co_name == fdef.name)
    return inner, sys.modules[__name__]


def _as_list(x):
    return x if isinstance(x, list) else [x]


def convert_function(fn):
    """The control-flow-converted twin of ``fn`` (a function or bound method); ``fn`` itself
    when it has nothing to convert, its source is unavailable, or its closure cannot be rebuilt.
    The twin runs in ``fn``'s own globals with ``fn``'s own closure cells."""
    bound = getattr(fn, '__self__', None) if inspect.ismethod(fn) else None
    func = fn.__func__ if bound is not None else fn
    if not inspect.isfunction(func):
        return fn
    try:
        r = _convert_code(func)
    except (OSError, TypeError, SyntaxError, IndentationError, StopIteration):
        return fn
    if r is None:
        return fn
    inner, jst = r
    cells = dict(zip(func.__code__.co_freevars, func.__closure__ or ()))
    closure = []
    for n in inner.co_freevars:
        if n == '_pra_jst':
            closure.append(types.CellType(jst))
        elif n in cells:
            closure.append(cells[n])
        else:  # (e.g. __class__ without the original's cell): keep the unconverted function
            return fn
    new = types.FunctionType(inner, func.__globals__, func.__name__, func.__defaults__, tuple(closure))
    new.__kwdefaults__ = func.__kwdefaults__
    new.__qualname__ = func.__qualname__
    new._pra_converted = True
    return types.MethodType(new, bound) if bound is not None else new
