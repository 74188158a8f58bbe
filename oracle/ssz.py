"""Minimal SSZ (SimpleSerialize) restatement — TEST INFRASTRUCTURE ONLY.

Restates the parts of upstream SSZ / remerkleable that the reference's light-client blocks
rely on (none of it lives in /root/reference; SURVEY.md §2 "[upstream] SSZ merkleization",
call sites `sync-protocol.md:191,212,354,357,427,444,463`):

  * basic types uint64/uint256, ByteVector[N] (Bytes4/20/32/48/96), ByteList[N],
    Vector[T, N], Bitvector[N], Container (field order = class annotation order);
  * `hash_tree_root` (merkleize with zero-subtree padding, `mix_in_length` for lists);
  * serialize / deserialize (fixed parts + 4-byte offsets for variable-size fields).

Containers are plain Python classes so the reference's own `class X(Container): ...` blocks
can be exec'd against this module (tests/golden/make_golden.py).
"""
from __future__ import annotations

import hashlib
import sys
from typing import Any, Dict, List, Tuple


# op counter (oracle/canonical.py): SHA-256 compressions of every sha256() call, ceil((len + 9) / 64)
SHA_COMPRESSIONS = [0]


def sha256(data: bytes) -> bytes:
    SHA_COMPRESSIONS[0] += (len(data) + 8) // 64 + 1
    return hashlib.sha256(data).digest()


ZERO_HASHES: List[bytes] = [bytes(32)]
for _ in range(64):
    ZERO_HASHES.append(sha256(ZERO_HASHES[-1] + ZERO_HASHES[-1]))
SHA_COMPRESSIONS[0] = 0  # the zero-subtree table is a constant, not per-call work


def _next_pow2_depth(n: int) -> int:
    return max(n - 1, 0).bit_length()


def merkleize(chunks: List[bytes], limit: int = None) -> bytes:
    n = len(chunks)
    if limit is None:
        limit = n
    assert n <= limit
    depth = _next_pow2_depth(limit)
    if n == 0:
        return ZERO_HASHES[depth]
    layer = list(chunks)
    for d in range(depth):
        if len(layer) % 2:
            layer.append(ZERO_HASHES[d])
        layer = [sha256(layer[i] + layer[i + 1]) for i in range(0, len(layer), 2)]
    return layer[0]


def mix_in_length(root: bytes, length: int) -> bytes:
    return sha256(root + length.to_bytes(32, "little"))


def pack_bytes(b: bytes) -> List[bytes]:
    if len(b) == 0:
        return []
    padded = b + bytes((-len(b)) % 32)
    return [padded[i:i + 32] for i in range(0, len(padded), 32)]


# ----------------------------------------------------------------------------- basic types
class uint64(int):
    SIZE = 8

    def __new__(cls, v: int = 0):
        v = int(v)
        if not 0 <= v < 2 ** 64:
            raise ValueError("uint64 out of range")
        return super().__new__(cls, v)

    @classmethod
    def default(cls):
        return cls(0)

    @classmethod
    def is_fixed(cls):
        return True

    @classmethod
    def fixed_size(cls):
        return cls.SIZE

    @classmethod
    def htr(cls, v) -> bytes:
        return int(v).to_bytes(32, "little")

    @classmethod
    def ser(cls, v) -> bytes:
        return int(v).to_bytes(cls.SIZE, "little")

    @classmethod
    def de(cls, b: bytes):
        if len(b) != cls.SIZE:
            raise ValueError("uint size")
        return cls(int.from_bytes(b, "little"))


class uint256(uint64):
    SIZE = 32

    def __new__(cls, v: int = 0):
        v = int(v)
        if not 0 <= v < 2 ** 256:
            raise ValueError("uint256 out of range")
        return int.__new__(cls, v)


class uint8(uint64):
    SIZE = 1

    def __new__(cls, v: int = 0):
        v = int(v)
        if not 0 <= v < 2 ** 8:
            raise ValueError("uint8 out of range")
        return int.__new__(cls, v)


class boolean(uint8):
    def __new__(cls, v: int = 0):
        v = int(v)
        if v not in (0, 1):
            raise ValueError("boolean is 0 or 1")
        return int.__new__(cls, v)


class _ByteVectorBase(bytes):
    LENGTH = 0

    def __new__(cls, v: bytes = None):
        if v is None:
            v = bytes(cls.LENGTH)
        v = bytes(v)
        if len(v) != cls.LENGTH:
            raise ValueError(f"{cls.__name__} needs {cls.LENGTH} bytes, got {len(v)}")
        return super().__new__(cls, v)

    @classmethod
    def default(cls):
        return cls()

    @classmethod
    def is_fixed(cls):
        return True

    @classmethod
    def fixed_size(cls):
        return cls.LENGTH

    @classmethod
    def htr(cls, v) -> bytes:
        chunks = pack_bytes(bytes(v))
        return merkleize(chunks, (cls.LENGTH + 31) // 32)

    @classmethod
    def ser(cls, v) -> bytes:
        return bytes(v)

    @classmethod
    def de(cls, b: bytes):
        return cls(b)


_BV_CACHE: Dict[int, type] = {}


class _ByteVectorFactory:
    def __getitem__(self, n: int) -> type:
        if n not in _BV_CACHE:
            _BV_CACHE[n] = type(f"ByteVector{n}", (_ByteVectorBase,), {"LENGTH": n})
        return _BV_CACHE[n]


ByteVector = _ByteVectorFactory()
Bytes4 = ByteVector[4]
Bytes20 = ByteVector[20]
Bytes32 = ByteVector[32]
Bytes48 = ByteVector[48]
Bytes96 = ByteVector[96]


class _ByteListBase(bytes):
    LIMIT = 0

    def __new__(cls, v: bytes = b""):
        v = bytes(v)
        if len(v) > cls.LIMIT:
            raise ValueError("ByteList over limit")
        return super().__new__(cls, v)

    @classmethod
    def default(cls):
        return cls()

    @classmethod
    def is_fixed(cls):
        return False

    @classmethod
    def htr(cls, v) -> bytes:
        return mix_in_length(merkleize(pack_bytes(bytes(v)), (cls.LIMIT + 31) // 32), len(v))

    @classmethod
    def ser(cls, v) -> bytes:
        return bytes(v)

    @classmethod
    def de(cls, b: bytes):
        return cls(b)


_BL_CACHE: Dict[int, type] = {}


class _ByteListFactory:
    def __getitem__(self, n: int) -> type:
        if n not in _BL_CACHE:
            _BL_CACHE[n] = type(f"ByteList{n}", (_ByteListBase,), {"LIMIT": n})
        return _BL_CACHE[n]


ByteList = _ByteListFactory()


def _type_of(t):
    return t


def _default_of(t):
    return t.default()


class _VectorBase(list):
    ELEM: Any = None
    LENGTH = 0

    def __init__(self, *args):
        if len(args) == 1 and not isinstance(args[0], (bytes, int)):
            items = list(args[0])
        elif len(args) == 0:
            items = [_default_of(self.ELEM) for _ in range(self.LENGTH)]
        else:
            items = list(args)
        if len(items) != self.LENGTH:
            raise ValueError(f"{type(self).__name__} needs {self.LENGTH} elements, got {len(items)}")
        super().__init__(self.ELEM(x) if not isinstance(x, self.ELEM) else x for x in items)

    @classmethod
    def default(cls):
        return cls()

    @classmethod
    def is_fixed(cls):
        return cls.ELEM.is_fixed()

    @classmethod
    def fixed_size(cls):
        return cls.ELEM.fixed_size() * cls.LENGTH

    @classmethod
    def htr(cls, v) -> bytes:
        if issubclass(cls.ELEM, uint64):  # basic: pack
            data = b"".join(cls.ELEM.ser(x) for x in v)
            return merkleize(pack_bytes(data), (cls.LENGTH * cls.ELEM.SIZE + 31) // 32)
        return merkleize([cls.ELEM.htr(x) for x in v], cls.LENGTH)

    @classmethod
    def ser(cls, v) -> bytes:
        assert cls.is_fixed()
        return b"".join(cls.ELEM.ser(x) for x in v)

    @classmethod
    def de(cls, b: bytes):
        sz = cls.ELEM.fixed_size()
        if len(b) != sz * cls.LENGTH:
            raise ValueError("Vector size")
        return cls([cls.ELEM.de(b[i * sz:(i + 1) * sz]) for i in range(cls.LENGTH)])


_V_CACHE: Dict[Tuple[Any, int], type] = {}


class _VectorFactory:
    def __getitem__(self, params) -> type:
        elem, n = params
        key = (elem, n)
        if key not in _V_CACHE:
            _V_CACHE[key] = type(f"Vector[{elem.__name__},{n}]", (_VectorBase,), {"ELEM": elem, "LENGTH": n})
        return _V_CACHE[key]


Vector = _VectorFactory()


class _ListBase(list):
    """List[T, N]: basic elements packed, composite elements by root; hash_tree_root mixes in the length."""
    ELEM: Any = None
    LIMIT = 0

    def __init__(self, items=()):
        items = list(items)
        if len(items) > self.LIMIT:
            raise ValueError(f"{type(self).__name__} over its limit")
        super().__init__(self.ELEM(x) if not isinstance(x, self.ELEM) else x for x in items)

    @classmethod
    def default(cls):
        return cls()

    @classmethod
    def is_fixed(cls):
        return False

    @classmethod
    def is_basic(cls):
        return issubclass(cls.ELEM, uint64)

    @classmethod
    def chunk_limit(cls):
        return (cls.LIMIT * cls.ELEM.SIZE + 31) // 32 if cls.is_basic() else cls.LIMIT

    @classmethod
    def data_root(cls, v) -> bytes:
        if cls.is_basic():
            return merkleize(pack_bytes(b"".join(cls.ELEM.ser(x) for x in v)), cls.chunk_limit())
        return merkleize([cls.ELEM.htr(x) for x in v], cls.LIMIT)

    @classmethod
    def htr(cls, v) -> bytes:
        return mix_in_length(cls.data_root(v), len(v))

    @classmethod
    def ser(cls, v) -> bytes:
        if cls.ELEM.is_fixed():
            return b"".join(cls.ELEM.ser(x) for x in v)
        parts = [cls.ELEM.ser(x) for x in v]
        off = 4 * len(parts)
        head = bytearray()
        for p in parts:
            head += off.to_bytes(4, "little")
            off += len(p)
        return bytes(head) + b"".join(parts)

    @classmethod
    def de(cls, b: bytes):
        if cls.ELEM.is_fixed():
            sz = cls.ELEM.fixed_size()
            if len(b) % sz:
                raise ValueError("List size")
            return cls([cls.ELEM.de(b[i:i + sz]) for i in range(0, len(b), sz)])
        if not b:
            return cls()
        first = int.from_bytes(b[:4], "little")
        if first % 4 or first > len(b):
            raise ValueError("List offsets")
        offs = [int.from_bytes(b[i:i + 4], "little") for i in range(0, first, 4)] + [len(b)]
        if any(offs[k + 1] < offs[k] for k in range(len(offs) - 1)):
            raise ValueError("List offsets")
        return cls([cls.ELEM.de(b[offs[k]:offs[k + 1]]) for k in range(len(offs) - 1)])


_L_CACHE: Dict[Tuple[Any, int], type] = {}


class _ListFactory:
    def __getitem__(self, params) -> type:
        elem, n = params
        key = (elem, n)
        if key not in _L_CACHE:
            _L_CACHE[key] = type(f"List[{elem.__name__},{n}]", (_ListBase,), {"ELEM": elem, "LIMIT": n})
        return _L_CACHE[key]


SSZList = _ListFactory()


class _BitvectorBase(list):
    LENGTH = 0

    def __init__(self, items=None):
        if items is None:
            items = [False] * self.LENGTH
        items = [bool(x) for x in items]
        if len(items) != self.LENGTH:
            raise ValueError("Bitvector length")
        super().__init__(items)

    @classmethod
    def default(cls):
        return cls()

    @classmethod
    def is_fixed(cls):
        return True

    @classmethod
    def fixed_size(cls):
        return (cls.LENGTH + 7) // 8

    @classmethod
    def ser(cls, v) -> bytes:
        out = bytearray(cls.fixed_size())
        for i, bit in enumerate(v):
            if bit:
                out[i // 8] |= 1 << (i % 8)
        return bytes(out)

    @classmethod
    def de(cls, b: bytes):
        if len(b) != cls.fixed_size():
            raise ValueError("Bitvector size")
        bits = [bool((b[i // 8] >> (i % 8)) & 1) for i in range(cls.LENGTH)]
        # unused high bits of the last byte must be zero
        if cls.LENGTH % 8 and b[-1] >> (cls.LENGTH % 8):
            raise ValueError("Bitvector padding")
        return cls(bits)

    @classmethod
    def htr(cls, v) -> bytes:
        return merkleize(pack_bytes(cls.ser(v)), (cls.LENGTH + 255) // 256)


_BITV_CACHE: Dict[int, type] = {}


class _BitvectorFactory:
    def __getitem__(self, n: int) -> type:
        if n not in _BITV_CACHE:
            _BITV_CACHE[n] = type(f"Bitvector{n}", (_BitvectorBase,), {"LENGTH": n})
        return _BITV_CACHE[n]


Bitvector = _BitvectorFactory()


class Container:
    """Field order = annotation order of the class body (as SSZ requires)."""

    _fields: List[Tuple[str, Any]] = []

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        fields = []
        for base in reversed(cls.__mro__[1:]):
            if issubclass(base, Container) and base is not Container:
                fields = list(base._fields)
        ann = cls.__dict__.get("__annotations__", {})
        mod = sys.modules.get(cls.__module__)
        scope = dict(vars(mod)) if mod is not None else {}
        for name, t in ann.items():
            if isinstance(t, str):  # `from __future__ import annotations` in the defining module
                t = eval(t, scope)
            fields.append((name, t))
        cls._fields = fields

    def __init__(self, **kwargs):
        for name, t in self._fields:
            if name in kwargs:
                v = kwargs.pop(name)
                if not isinstance(v, t):
                    v = t(v)
                object.__setattr__(self, name, v)
            else:
                object.__setattr__(self, name, t.default())
        if kwargs:
            raise TypeError(f"unknown fields {list(kwargs)}")

    def __setattr__(self, name, value):
        for fname, t in self._fields:
            if fname == name:
                if not isinstance(value, t):
                    value = t(value)
                object.__setattr__(self, name, value)
                return
        raise AttributeError(name)

    def __eq__(self, other):
        if type(self) is not type(other):
            return NotImplemented
        return all(getattr(self, n) == getattr(other, n) for n, _ in self._fields)

    def __ne__(self, other):
        r = self.__eq__(other)
        return r if r is NotImplemented else not r

    def __repr__(self):
        return f"{type(self).__name__}(" + ", ".join(f"{n}={getattr(self, n)!r}" for n, _ in self._fields) + ")"

    def copy(self):
        return type(self).de(type(self).ser(self))

    @classmethod
    def default(cls):
        return cls()

    @classmethod
    def is_fixed(cls):
        return all(t.is_fixed() for _, t in cls._fields)

    @classmethod
    def fixed_size(cls):
        assert cls.is_fixed()
        return sum(t.fixed_size() for _, t in cls._fields)

    @classmethod
    def htr(cls, v) -> bytes:
        return merkleize([t.htr(getattr(v, n)) for n, t in cls._fields])

    @classmethod
    def ser(cls, v) -> bytes:
        fixed_parts, var_parts = [], []
        for n, t in cls._fields:
            if t.is_fixed():
                fixed_parts.append(t.ser(getattr(v, n)))
                var_parts.append(b"")
            else:
                fixed_parts.append(None)
                var_parts.append(t.ser(getattr(v, n)))
        fixed_len = sum(4 if p is None else len(p) for p in fixed_parts)
        out = bytearray()
        off = fixed_len
        for p, vp in zip(fixed_parts, var_parts):
            if p is None:
                out += off.to_bytes(4, "little")
                off += len(vp)
            else:
                out += p
        for vp in var_parts:
            out += vp
        return bytes(out)

    @classmethod
    def de(cls, b: bytes):
        pos = 0
        vals: Dict[str, Any] = {}
        offsets = []
        for n, t in cls._fields:
            if t.is_fixed():
                sz = t.fixed_size()
                if pos + sz > len(b):
                    raise ValueError("container truncated")
                vals[n] = t.de(b[pos:pos + sz])
                pos += sz
            else:
                if pos + 4 > len(b):
                    raise ValueError("container truncated")
                offsets.append((n, t, int.from_bytes(b[pos:pos + 4], "little")))
                pos += 4
        if offsets:
            if offsets[0][2] != pos:
                raise ValueError("first offset mismatch")
            for k, (n, t, o) in enumerate(offsets):
                end = offsets[k + 1][2] if k + 1 < len(offsets) else len(b)
                if end < o or end > len(b):
                    raise ValueError("bad offsets")
                vals[n] = t.de(b[o:end])
        elif pos != len(b):
            raise ValueError("trailing bytes")
        return cls(**vals)


def hash_tree_root(value) -> bytes:
    t = type(value)
    if hasattr(t, "htr"):
        return Bytes32(t.htr(value))
    raise TypeError(f"no SSZ type for {t}")


def serialize(value) -> bytes:
    return type(value).ser(value)


# ----------------------------------------------------------------------------- Merkle proofs
def _tree_path(chunks: List[bytes], depth: int, idx: int) -> List[bytes]:
    """Sibling roots on the path to leaf idx of merkleize(chunks) padded to 2^depth, bottom-up."""
    out = []
    layer = list(chunks)
    for d in range(depth):
        sib = idx ^ 1
        out.append(layer[sib] if sib < len(layer) else ZERO_HASHES[d])
        if len(layer) % 2:
            layer.append(ZERO_HASHES[d])
        layer = [sha256(layer[i] + layer[i + 1]) for i in range(0, len(layer), 2)]
        idx >>= 1
    return out


def compute_merkle_proof(obj, gindex: int) -> List[bytes]:
    """The Merkle branch of the node at generalized index `gindex` inside SSZ object `obj` (bottom-up,
    the order is_valid_merkle_branch consumes).  Restates the upstream helper the reference declares
    without a body (full-node.md:35-38) for the containers / vectors / lists of this module."""
    bits = bin(int(gindex))[3:]
    node, levels = obj, []
    while bits:
        t = type(node)
        if isinstance(node, _ListBase):          # root = H(data_root, length)
            if bits[0] == "1":
                levels.append([t.data_root(node)])
                assert len(bits) == 1, "nothing below a list's length chunk"
                bits = ""
                continue
            levels.append([len(node).to_bytes(32, "little")])
            bits = bits[1:]
            assert not t.is_basic(), "proofs into packed basic lists are not needed here"
            depth = _next_pow2_depth(t.LIMIT)
            children, chunks = list(node), [t.ELEM.htr(x) for x in node]
        elif isinstance(node, Container):
            depth = _next_pow2_depth(len(t._fields))
            children = [getattr(node, n) for n, _ in t._fields]
            chunks = [ft.htr(c) for c, (_, ft) in zip(children, t._fields)]
        elif isinstance(node, _VectorBase) and not issubclass(t.ELEM, uint64):
            depth = _next_pow2_depth(t.LENGTH)
            children, chunks = list(node), [t.ELEM.htr(x) for x in node]
        else:
            raise TypeError(f"no Merkle descent into {t.__name__}")
        take, bits = bits[:depth], bits[depth:]
        assert len(take) == depth, "generalized index ends inside a subtree"
        idx = int(take, 2) if take else 0
        levels.append(_tree_path(chunks, depth, idx))
        node = children[idx] if idx < len(children) else None
        assert node is not None or not bits
    out = []
    for lv in reversed(levels):
        out += lv
    return out
