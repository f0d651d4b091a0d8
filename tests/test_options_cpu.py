"""The library's developer options (tsdbhip_set_option) and its independence from the process
environment: no getenv anywhere in the library sources, no TSDBHIP_* name in the built library,
every option named in opts.h settable by name, unknown names refused.  (No GPU needed.)"""
from __future__ import annotations

import os
import re

import pytest

from opentsdb_amd import abi
from opentsdb_amd import engine as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "opentsdb_amd", "csrc")


def test_no_getenv_in_library_sources():
    hits = []
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".cpp", ".h", ".hip")):
            for i, ln in enumerate(open(os.path.join(CSRC, f)), 1):
                if re.search(r"\bgetenv\s*\(|\bsecure_getenv\s*\(|\benviron\b", ln):
                    hits.append(f"{f}:{i}")
    assert not hits, hits


def test_no_environment_switch_names_in_the_built_library():
    # (the getenv the library imports is rocPRIM's own ROCPRIM_USE_ATOMIC_BLOCK_ID, read inside the
    # hipcub scans it instantiates: rocprim/device/detail/ordered_block_id.hpp)
    data = open(E.LIB_PATH, "rb").read()
    assert b"TSDBHIP_" not in data


def test_option_table_matches_opts_h():
    names = re.findall(r"^\s*OPT_([A-Z0-9_]+),", open(os.path.join(CSRC, "opts.h")).read(), re.M)
    names = [n for n in names if n != "COUNT"]
    assert names == E.OPTIONS
    hdr = open(os.path.join(ROOT, "include", "tsdbhip.h")).read()
    for n in names:
        assert n in hdr


def test_set_get_reset():
    try:
        for n in E.OPTIONS:
            assert E.get_option(n) == -1
        E.set_option("SEL_WIN", 2)
        assert E.get_option("SEL_WIN") == 2
        with E.options(FAST=0, HWIN=0):
            assert E.get_option("FAST") == 0 and E.get_option("HWIN") == 0
        assert E.get_option("FAST") == -1 and E.get_option("HWIN") == -1
        E.set_option("SEL_WIN", None)
        assert E.get_option("SEL_WIN") == -1
    finally:
        E.reset_options()


@pytest.mark.parametrize("name", ["TSDBHIP_FAST", "fast", "", "SEL_T", "HIST_DBG", "PULL"])
def test_unknown_or_removed_options_refused(name):
    with pytest.raises(E.EngineError) as ei:
        E.set_option(name, 1)
    assert ei.value.code == abi.TSDB_E_ILLEGAL_ARGUMENT


def test_negative_values_refused():
    with pytest.raises(E.EngineError):
        E.set_option("FAST", -2)
