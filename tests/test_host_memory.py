"""Host memory budget of the store pipeline (host_available_bytes, host/zt_store.cpp and
store.py): MemAvailable capped by a memory-limited cgroup's limit minus its usage, the usage net
of reclaimable (inactive) page cache, read through fake /proc and cgroup files."""
import os

import pytest

from zarrs_tools_amd import _abi
from zarrs_tools_amd import store as S

GIB = 1 << 30


def _write(path, text):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(text)


@pytest.fixture
def fake_root(tmp_path, monkeypatch):
    monkeypatch.delenv("ZT_STORE_HOST_MEMORY", raising=False)
    _write(str(tmp_path / "meminfo"), f"MemTotal: {64 * GIB // 1024} kB\n"
           f"MemAvailable: {40 * GIB // 1024} kB\n")
    monkeypatch.setenv("ZT_MEMINFO", str(tmp_path / "meminfo"))
    monkeypatch.setenv("ZT_CGROUP_ROOT", str(tmp_path / "cg"))
    return tmp_path


def _both():
    return S.host_available_bytes(), int(_abi.lib().zt_store_host_available_bytes())


def test_no_cgroup_limit_uses_memavailable(fake_root):
    assert _both() == (40 * GIB, 40 * GIB)
    _write(str(fake_root / "cg" / "memory.max"), "max\n")
    _write(str(fake_root / "cg" / "memory.current"), f"{10 * GIB}\n")
    assert _both() == (40 * GIB, 40 * GIB)


def test_cgroup_v2_page_cache_counts_as_available(fake_root):
    cg = fake_root / "cg"
    _write(str(cg / "memory.max"), f"{32 * GIB}\n")
    # 31 GiB charged, 20 GiB of it inactive file cache: 32 - (31 - 20) = 21 GiB available
    _write(str(cg / "memory.current"), f"{31 * GIB}\n")
    _write(str(cg / "memory.stat"), f"anon {10 * GIB}\nfile {21 * GIB}\n"
           f"active_file {1 * GIB}\ninactive_file {20 * GIB}\n")
    assert _both() == (21 * GIB, 21 * GIB)
    # without memory.stat: limit minus the raw usage
    os.remove(str(cg / "memory.stat"))
    assert _both() == (1 * GIB, 1 * GIB)


def test_cgroup_v1_total_inactive_file(fake_root):
    cg = fake_root / "cg" / "memory"
    _write(str(cg / "memory.limit_in_bytes"), f"{16 * GIB}\n")
    _write(str(cg / "memory.usage_in_bytes"), f"{15 * GIB}\n")
    _write(str(cg / "memory.stat"), f"cache {12 * GIB}\ninactive_file {1}\n"
           f"total_inactive_file {10 * GIB}\n")
    assert _both() == (11 * GIB, 11 * GIB)


def test_memavailable_still_bounds_a_large_cgroup(fake_root):
    cg = fake_root / "cg"
    _write(str(cg / "memory.max"), f"{200 * GIB}\n")
    _write(str(cg / "memory.current"), f"{1 * GIB}\n")
    assert _both() == (40 * GIB, 40 * GIB)


def test_env_override(fake_root, monkeypatch):
    monkeypatch.setenv("ZT_STORE_HOST_MEMORY", str(3 * GIB))
    assert _both() == (3 * GIB, 3 * GIB)
