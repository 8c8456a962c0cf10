"""The C-ABI library loads on a CPU host and exports every function include/*.h declares."""
import ctypes
import os
import re

from tigerbeetle_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set()
    for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b((?:tbg|tbr|tb_sm|tb_multi_batch)_\w+)\s*\(", text,
                         flags=re.M):
        names.add(m.group(1))
    return names


def test_headers_declare_the_bound_symbols():
    declared = (declared_functions("tbg.h") | declared_functions("tb_state_machine.h") |
                declared_functions("tbr.h") | declared_functions("tbg_group.h"))
    bound = {name for name, _, _ in native.SIGNATURES}
    assert declared == bound, (declared - bound, bound - declared)


def test_library_exports_every_declared_symbol():
    lib = native.load()
    for name in (declared_functions("tbg.h") | declared_functions("tb_state_machine.h") |
                 declared_functions("tbr.h") | declared_functions("tbg_group.h")):
        assert hasattr(lib, name), name


def test_struct_sizes():
    from tigerbeetle_amd.types import ACCOUNT_DTYPE, RESULT_DTYPE, TRANSFER_DTYPE
    assert ACCOUNT_DTYPE.itemsize == 128 and TRANSFER_DTYPE.itemsize == 128
    assert RESULT_DTYPE.itemsize == 16
    assert ctypes.sizeof(native.TbgOptions) == 48
    assert ctypes.sizeof(native.Executor) == 12 * 8
    from tigerbeetle_amd.types import (ACCOUNT_EVENT_DTYPE, CHANGE_EVENT_DTYPE,
                                       CHANGE_EVENTS_FILTER_DTYPE)
    assert ACCOUNT_EVENT_DTYPE.itemsize == 256 and CHANGE_EVENT_DTYPE.itemsize == 384
    assert CHANGE_EVENTS_FILTER_DTYPE.itemsize == 64
    from tigerbeetle_amd.types import (ACCOUNT_BALANCE_DTYPE, ACCOUNT_FILTER_DTYPE,
                                       QUERY_FILTER_DTYPE)
    assert ACCOUNT_FILTER_DTYPE.itemsize == 128 and QUERY_FILTER_DTYPE.itemsize == 64
    assert ACCOUNT_BALANCE_DTYPE.itemsize == 128
    assert ACCOUNT_FILTER_DTYPE.fields["timestamp_min"][1] == 104
    assert QUERY_FILTER_DTYPE.fields["timestamp_min"][1] == 40
