"""CPU-side checks of the product boundary: the C-ABI library loads and exports every symbol that
include/zb_engine.h declares (no compute calls: there is no GPU in the build container)."""
import ctypes
import os
import re

from zeebe_amd import engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "zb_engine.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|void\*|void|const char\*)\s*(zb_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_api():
    syms = declared_symbols()
    assert set(syms) == set(engine.EXPORTED_SYMBOLS), syms


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(engine.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(lib, s), s


def test_config_flags_match_header():
    """Every ZB_CFG_* flag of include/zb_engine.h has the same value as engine.CFG_* (the Python binding's copy)."""
    src = open(os.path.join(ROOT, "include", "zb_engine.h")).read()
    flags = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define ZB_CFG_(\w+)\s+(\d+)", src)}
    assert flags and "RCCL_SELF" in flags, flags
    for name, value in flags.items():
        assert getattr(engine, "CFG_" + name) == value, name
    assert len(set(flags.values())) == len(flags)  # (distinct bits)


def test_config_struct_layout_matches_header():
    assert ctypes.sizeof(engine.zb_config) == 48
    assert ctypes.sizeof(engine.zb_rec) == 32
    assert ctypes.sizeof(engine.zb_record_header) == 24


def test_workloads_payload_encoding():
    import msgpack

    from zeebe_amd import workloads

    blob, offs = workloads.order_payloads(300)
    docs = workloads.split(blob, offs)
    assert [msgpack.unpackb(d) for d in docs] == [{"orderId": i} for i in range(300)]
    blob, offs = workloads.xor_payloads(50)
    for d in workloads.split(blob, offs):
        v = msgpack.unpackb(d, raw=False)
        assert 0 <= v["amount"] < 2000 and v["region"] in workloads.REGIONS and 0 <= v["score"] < 1
