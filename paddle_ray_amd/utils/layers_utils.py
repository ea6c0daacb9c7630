"""Nested-structure helpers (parity: python/paddle/utils/layers_utils.py flatten /
pack_sequence_as / map_structure / assert_same_structure). Sequences are lists/tuples
(namedtuples keep their type); dicts are walked in sorted-key order; anything else is a leaf."""


def is_sequence(seq):
    return isinstance(seq, (list, tuple, dict))


def _children(s):
    if isinstance(s, dict):
        return [s[k] for k in sorted(s)]
    return list(s)


def flatten(nest):
    if not is_sequence(nest):
        return [nest]
    out = []
    for c in _children(nest):
        out.extend(flatten(c))
    return out


def _rebuild(like, items):
    if isinstance(like, dict):
        return type(like)((k, v) for k, v in zip(sorted(like), items))
    if isinstance(like, tuple) and hasattr(like, '_fields'):  # namedtuple
        return type(like)(*items)
    return type(like)(items)


def pack_sequence_as(structure, flat_sequence):
    flat = list(flat_sequence)
    if not is_sequence(structure):
        if len(flat) != 1:
            raise ValueError(f"structure is a scalar but {len(flat)} values were given")
        return flat[0]
    pos = [0]

    def build(s):
        if not is_sequence(s):
            v = flat[pos[0]]
            pos[0] += 1
            return v
        return _rebuild(s, [build(c) for c in _children(s)])
    out = build(structure)
    if pos[0] != len(flat):
        raise ValueError(f"structure has {pos[0]} leaves but {len(flat)} values were given")
    return out


def assert_same_structure(nest1, nest2, check_types=True):
    if is_sequence(nest1) != is_sequence(nest2):
        raise ValueError(f"structures differ: {type(nest1)} vs {type(nest2)}")
    if not is_sequence(nest1):
        return
    if check_types and type(nest1) is not type(nest2):
        raise TypeError(f"structures differ: {type(nest1)} vs {type(nest2)}")
    c1, c2 = _children(nest1), _children(nest2)
    if len(c1) != len(c2):
        raise ValueError(f"structures differ in length: {len(c1)} vs {len(c2)}")
    for a, b in zip(c1, c2):
        assert_same_structure(a, b, check_types)


def map_structure(func, *structure):
    for s in structure[1:]:
        assert_same_structure(structure[0], s, check_types=False)
    flats = [flatten(s) for s in structure]
    return pack_sequence_as(structure[0], [func(*xs) for xs in zip(*flats)])
