"""distml_amd — MI355X-native parameter-server push path for DistML.

The product is libdistml_ps.so (include/distml_ps.h): HBM-resident DataStore
shards and HIP kernels for gfx950. This package is the host-side mirror of the
reference's DataStore plugin interface over that C-ABI.
"""
from ._lib import NativeLibraryMissing, load as load_library  # noqa: F401
from .datadesc import ALL, EMPTY, DataDesc, KeyCollection, KeyList, KeyRange  # noqa: F401
from .store import (ArrayIndexOutOfBoundsException, DataStore, DistMLException, DMatrix,  # noqa: F401
                    IllegalArgumentException, IllegalStateException, Model, NativeError,
                    encode_array_push, encode_matrix_push, pinned_empty)

__version__ = "0.1.0"
