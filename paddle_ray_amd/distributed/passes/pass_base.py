"""Program passes: registry, context and manager (parity: python/paddle/distributed/passes/
pass_base.py -- PassContext :20, PassType :42, PassBase :50, register_pass :124, new_pass :133,
the common conflict rules :170-269 and PassManager :352 with auto_solve_conflict).

A pass rewrites one or more ``paddle.static`` Programs in place. Passes here work on this
framework's own program IR (static/graph.py OpDescs): the distributed ones record their setting
in ``program._pass_cfg`` and rebuild the training part of an already-minimized program
(static/graph.py ``rebuild_training``); the fusion ones replace forward op patterns with the
in-tree HIP kernels' fused ops (static/fn_ops.py).

Conflict resolution (``PassManager(auto_solve_conflict=True)``): passes whose ``_check_self``
fails, or that conflict with a pass already applied in the context, are dropped; the rest keep
their given order except that fusion passes move behind every other pass, in the canonical
fusion order; then each pass that conflicts with one kept before it is dropped. (The
reference finds a longest conflict-free path over the pairwise rules; for the rule set below --
same-type, fusion-last, fusion-order, white lists -- the ordered greedy walk keeps the same
passes.)"""

__all__ = ['PassContext', 'PassType', 'PassBase', 'register_pass', 'new_pass', 'PassManager']


class PassContext:
    """Attributes shared between passes of one application plus the passes applied so far."""

    def __init__(self):
        self._applied = []
        self._attrs = {}

    def set_attr(self, key, value):
        self._attrs[key] = value

    def get_attr(self, key, default=None):
        return self._attrs.get(key, default)

    @property
    def passes(self):
        return self._applied

    def _add_pass(self, p):
        self._applied.append(p)

    def _pop_pass(self):
        self._applied.pop()


class PassType:
    UNKNOWN = 0
    COMM_OPT = 1
    CALC_OPT = 2
    PARALLEL_OPT = 3
    FUSION_OPT = 4


_REGISTRY = {}

# fusion passes run last, in this order (a fused op must not be split again by a later fusion)
FUSION_ORDER = ['fuse_relu_depthwise_conv', 'fuse_bn_add_act', 'fuse_bn_act', 'fused_attention',
                'fused_feedforward', 'fuse_gemm_epilogue', 'fuse_elewise_add_act', 'fuse_optimizer']

# (k, [v...]): k may be applied before any of v although a common rule would refuse it
BEFORE_WHITE_LISTS = {'fuse_gradient_merge': ['fuse_all_reduce']}
AFTER_WHITE_LISTS = {}


class PassBase:
    """One program rewrite. Subclasses implement ``_apply_single_impl(main, startup, context)``
    and may override ``_check_self`` (attributes valid?), ``_check_conflict(other)`` (can this
    pass run after ``other``?) and ``_type``."""
    name = None

    def __init__(self):
        self._attrs = {}

    def set_attr(self, key, value):
        self._attrs[key] = value
        return self

    def get_attr(self, key, default=None):
        return self._attrs.get(key, default)

    def _check_self(self):
        return True

    def _check_conflict(self, other_pass):
        return True

    def _type(self):
        return PassType.UNKNOWN

    def _compatible_after(self, before):
        """May this pass run after ``before``? Its own rule plus the common ones."""
        return self._check_conflict(before) and all(rule(before, self) for rule in _COMMON_RULES)

    # (reference name)
    _check_conflict_including_common_rules = _compatible_after

    def apply(self, main_programs, startup_programs=None, context=None):
        context = PassContext() if context is None else context
        mains = list(main_programs) if isinstance(main_programs, (list, tuple)) else [main_programs]
        if startup_programs is None:
            startups = [None] * len(mains)
        else:
            startups = list(startup_programs) if isinstance(startup_programs, (list, tuple)) \
                else [startup_programs]
        if len(mains) != len(startups):
            raise ValueError(f"{len(mains)} main programs but {len(startups)} startup programs")
        if not self._check_self():
            return context
        if not all(self._compatible_after(p) for p in context.passes):
            return context
        self._apply_impl(mains, startups, context)
        context._add_pass(self)
        return context

    def _apply_impl(self, mains, startups, context):
        for m, s in zip(mains, startups):
            self._apply_single_impl(m, s, context)

    def _apply_single_impl(self, main_program, startup_program, context):
        raise NotImplementedError

    def __repr__(self):
        return f"{type(self).__name__}({self.name!r}, {self._attrs})"


def register_pass(name):
    def deco(cls):
        if not (isinstance(cls, type) and issubclass(cls, PassBase)):
            raise TypeError(f"register_pass({name!r}) needs a PassBase subclass")
        _REGISTRY[name] = cls
        cls.name = name
        return cls
    return deco


def new_pass(name, pass_attrs=None):
    """An instance of the pass registered as ``name`` with ``pass_attrs`` set."""
    cls = _REGISTRY.get(name)
    if cls is None:
        raise AssertionError(f"Pass {name} is not registered (known: {sorted(_REGISTRY)})")
    p = cls()
    for k, v in (pass_attrs or {}).items():
        p.set_attr(k, v)
    return p


def registered_passes():
    return sorted(_REGISTRY)


# -- common conflict rules (before, after) -> may `after` follow `before`? ----------------------
def _fusion_last(before, after):
    return not (before._type() == PassType.FUSION_OPT and after._type() != PassType.FUSION_OPT)


def _fusion_index(p):
    return FUSION_ORDER.index(p.name) if p.name in FUSION_ORDER else len(FUSION_ORDER)


def _fusion_order(before, after):
    if before._type() == PassType.FUSION_OPT and after._type() == PassType.FUSION_OPT:
        return _fusion_index(before) < _fusion_index(after)
    return True


def _not_twice(before, after):
    return type(before) is not type(after)


def _white_lists(before, after):
    allowed = {}
    for k, vs in BEFORE_WHITE_LISTS.items():
        allowed.setdefault(k, set()).update(vs)
    for k, vs in AFTER_WHITE_LISTS.items():
        for v in vs:
            allowed.setdefault(v, set()).add(k)
    names = set(allowed) | {v for vs in allowed.values() for v in vs}
    if before.name not in allowed or after.name not in names:
        return True
    return after.name in allowed[before.name]


_COMMON_RULES = [_fusion_last, _fusion_order, _not_twice, _white_lists]


def _solve_conflicts(passes, context):
    cands = [p for p in passes if p._check_self()]
    cands = [p for p in cands if all(p._compatible_after(a) for a in context.passes)]
    plain = [p for p in cands if p._type() != PassType.FUSION_OPT]
    fusion = sorted((p for p in cands if p._type() == PassType.FUSION_OPT), key=_fusion_index)
    kept = []
    for p in plain + fusion:
        if all(p._compatible_after(k) for k in kept):
            kept.append(p)
    return kept


class PassManager:
    """Apply a list of passes in order (``auto_solve_conflict``: drop / reorder as described in
    the module docstring)."""

    def __init__(self, passes, context=None, auto_solve_conflict=True):
        self._context = PassContext() if context is None else context
        self._passes = _solve_conflicts(list(passes), self._context) if auto_solve_conflict \
            else list(passes)

    def apply(self, main_programs, startup_programs=None):
        ctx = self._context
        for p in self._passes:
            ctx = p.apply(main_programs, startup_programs, ctx)
        self._context = ctx
        return ctx

    @property
    def context(self):
        return self._context

    @property
    def names(self):
        return [p.name for p in self._passes]

    @property
    def passes(self):
        return tuple(self._passes)
