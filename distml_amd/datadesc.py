"""DataDesc and the key collections of DistML's wire format, restated for the host.

DataDesc          <- src/main/java/com/intel/distml/util/DataDesc.java:8-245
KeyCollection     <- util/KeyCollection.java (intersect :76-95)
KeyRange          <- util/KeyRange.java (linearSplit :68-80, intersect :123-144)
KeyList           <- util/KeyList.java (iteration = the caller's insertion order here;
                     Java's HashSet order is not reproduced)
"""
from __future__ import annotations

import struct
from typing import Iterable, Iterator, List

from ._lib import dml_desc


class DataDesc:
    DATA_TYPE_ARRAY = 0
    DATA_TYPE_MATRIX = 1
    KEY_TYPE_INT = 0
    KEY_TYPE_LONG = 1
    ELEMENT_TYPE_INT = 0
    ELEMENT_TYPE_FLOAT = 1
    ELEMENT_TYPE_LONG = 2
    ELEMENT_TYPE_DOUBLE = 3

    def __init__(self, dataType, keyType, valueType, denseRow=False, denseColumn=True, adaGrad=False):
        # DataDesc.java:35-52
        self.dataType = dataType
        self.keyType = keyType
        self.valueType = valueType
        self.denseRow = bool(denseRow)
        self.denseColumn = bool(denseColumn)
        self.adaGrad = bool(adaGrad)
        self.keySize = 4 if keyType == self.KEY_TYPE_INT else 8
        self.valueSize = 4 if valueType in (self.ELEMENT_TYPE_INT, self.ELEMENT_TYPE_FLOAT) else 8

    def to_c(self) -> dml_desc:
        return dml_desc(self.dataType, self.keyType, self.valueType, int(self.denseRow),
                        int(self.denseColumn), int(self.adaGrad))

    def write(self) -> bytes:
        """Six big-endian ints, DataDesc.write (DataDesc.java:62-69)."""
        return struct.pack(">6i", self.dataType, self.keyType, self.valueType, int(self.denseRow),
                           int(self.denseColumn), int(self.adaGrad))

    @classmethod
    def read(cls, buf: bytes) -> "DataDesc":
        d = struct.unpack(">6i", buf[:24])
        return cls(d[0], d[1], d[2], d[3] == 1, d[4] == 1, d[5] == 1)

    def same_layout(self, other: "DataDesc") -> bool:
        return (self.dataType, self.keyType, self.valueType, self.denseColumn, self.adaGrad) == \
               (other.dataType, other.keyType, other.valueType, other.denseColumn, other.adaGrad)

    def __repr__(self):
        return f"{self.dataType}, {self.keyType}, {self.keySize}, {self.valueType}, {self.valueSize}"


class KeyCollection:
    TYPE_ALL, TYPE_EMPTY, TYPE_RANGE, TYPE_LIST, TYPE_HASH = 0, 1, 2, 3, 4

    def contains(self, key: int) -> bool:
        raise NotImplementedError

    def __iter__(self) -> Iterator[int]:
        raise NotImplementedError

    def size(self) -> int:
        raise NotImplementedError

    def isEmpty(self) -> bool:
        return self.size() == 0

    def intersect(self, keys: "KeyCollection") -> "KeyCollection":
        # KeyCollection.intersect (KeyCollection.java:76-95)
        if isinstance(keys, AllKeys):
            return self
        if isinstance(keys, EmptyKeys):
            return keys
        return KeyList(k for k in keys if self.contains(k))


class EmptyKeys(KeyCollection):
    def contains(self, key):
        return False

    def __iter__(self):
        return iter(())

    def size(self):
        return 0

    def intersect(self, keys):
        return self


class AllKeys(KeyCollection):
    def contains(self, key):
        return True

    def __iter__(self):
        raise TypeError("This is an ALL_KEYS instance, not iterable.")

    def size(self):
        raise TypeError("This is an ALL_KEYS instance, size unknown")

    def intersect(self, keys):
        return keys


EMPTY = EmptyKeys()
ALL = AllKeys()


class KeyRange(KeyCollection):
    def __init__(self, firstKey: int, lastKey: int):
        self.firstKey = int(firstKey)
        self.lastKey = int(lastKey)

    def __eq__(self, other):
        return isinstance(other, KeyRange) and (self.firstKey, self.lastKey) == (other.firstKey, other.lastKey)

    def __hash__(self):
        return hash((self.firstKey, self.lastKey))

    def linearSplit(self, hostNum: int) -> List["KeyRange"]:
        # KeyRange.java:68-80 (Java long division truncates toward zero)
        start = self.firstKey
        num = self.lastKey - self.firstKey + hostNum
        step = abs(num) // hostNum * (1 if num >= 0 else -1)
        out = []
        for _ in range(hostNum):
            end = min(start + step - 1, self.lastKey)
            out.append(KeyRange(start, end))
            start += step
        return out

    def size(self) -> int:
        return self.lastKey - self.firstKey + 1

    def contains(self, key: int) -> bool:
        return self.firstKey <= key <= self.lastKey

    def isEmpty(self) -> bool:
        return self.firstKey > self.lastKey

    def __iter__(self):
        return iter(range(self.firstKey, self.lastKey + 1))

    def intersect(self, keys: KeyCollection) -> KeyCollection:
        # KeyRange.java:123-144
        if isinstance(keys, KeyRange):
            lo, hi = max(keys.firstKey, self.firstKey), min(keys.lastKey, self.lastKey)
            return EMPTY if lo > hi else KeyRange(lo, hi)
        return super().intersect(keys)

    def __repr__(self):
        return f"[{self.firstKey}, {self.lastKey}]"


class KeyList(KeyCollection):
    def __init__(self, keys: Iterable[int] = ()):
        self.keys = list(dict.fromkeys(int(k) for k in keys))  # a set, in insertion order

    def addKey(self, k: int):
        if k not in self.keys:
            self.keys.append(int(k))

    def contains(self, key):
        return key in set(self.keys)

    def __iter__(self):
        return iter(self.keys)

    def size(self):
        return len(self.keys)

    def intersect(self, keys):
        mine = set(self.keys)
        return KeyList(k for k in keys if k in mine)

    def __repr__(self):
        return f"[KeyList: size={len(self.keys)}]"
