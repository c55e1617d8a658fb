"""Code-object checks of the memory ordering the xGMI schedule relies on
(csrc/ono_device.h): a deterministic test, no GPU needed.

Stores that another rank reads after a flag barrier — the push into a peer's
receive slot, the owner chain's result slot / peer gather slots, the PS shard
copy — must be system-coherent (`global_store… sc0 sc1`) and must be
acknowledged before the wave that issued them ends: nothing at a kernel
boundary waits for stores bound to another device's memory, and the barrier's
release fence runs in a later launch.  The race this prevents (an owner chain
reading a receive slot before the pushed slice landed) showed up about one run
in two before the waits existed, and can only be provoked by timing, so the
property is checked where it is decided: in the gfx950 code object shipped in
libono_reduce.so.  The check fails if the stores lose their system scope, or
if a wave can reach `s_endpgm` (or leave its block) with such a store not yet
waited for by `s_waitcnt vmcnt(0)`.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oxidized-neural-orchestra_amd", "ono_amd", "libono_reduce.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

pytestmark = pytest.mark.skipif(not (os.path.exists(LIB) and os.access(OBJDUMP, os.X_OK)),
                                reason="library or llvm-objdump missing")

_FUNC = re.compile(r"^[0-9a-f]+ <([^>]+)>:")


def _kernels(tmp_path) -> dict:
    """kernel symbol -> list of instruction strings (layout order), every
    gfx950 bundle of the library."""
    lib = tmp_path / "lib.so"
    shutil.copy(LIB, lib)
    subprocess.run([OBJDUMP, "--offloading", str(lib)], check=True, cwd=tmp_path, capture_output=True)
    out: dict = {}
    for f in sorted(os.listdir(tmp_path)):
        if "amdgcn" not in f or "gfx950" not in f:
            continue
        asm = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", str(tmp_path / f)], check=True,
                             capture_output=True, text=True).stdout
        cur = None
        for line in asm.splitlines():
            m = _FUNC.match(line)
            if m:
                cur = out.setdefault(m.group(1), [])
                continue
            ins = line.split("//")[0].strip()
            if cur is not None and ins:
                cur.append(ins)
    assert out, "no gfx950 code object found in libono_reduce.so"
    return out


def _is_sys_store(ins: str) -> bool:
    return ins.startswith(("global_store", "buffer_store", "flat_store")) and " sc0" in ins and " sc1" in ins


def _waits_vm0(ins: str) -> bool:
    return ins.startswith("s_waitcnt") and "vmcnt(0)" in ins


def _unwaited(instrs: list) -> list:
    """sys stores not followed by vmcnt(0) before the next s_endpgm / branch in layout order"""
    bad = []
    for i, ins in enumerate(instrs):
        if not _is_sys_store(ins):
            continue
        for nxt in instrs[i + 1:]:
            if _waits_vm0(nxt):
                break
            if nxt.startswith(("s_endpgm", "s_branch", "s_cbranch", "s_setpc")):
                bad.append(f"{ins!r} reaches {nxt!r} without s_waitcnt vmcnt(0)")
                break
        else:
            bad.append(f"{ins!r} is never waited for")
    return bad


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    return _kernels(tmp_path_factory.mktemp("isa"))


@pytest.mark.parametrize("op", ["PushOp", "DirectOp", "OptOp"])
def test_peer_visible_stores_are_system_scope(kernels, op):
    """every kernel that writes memory peers read has sc0 sc1 stores (push
    always; DirectOp with sys_out and OptOp with the PS fence, run-time flags
    compiled into the same kernel)"""
    ks = {k: v for k, v in kernels.items() if op in k}
    assert ks, f"no {op} kernel in the code object"
    missing = [k for k, v in ks.items() if not any(_is_sys_store(i) for i in v)]
    assert not missing, f"{op} kernels without system-scope stores: {missing[:3]}"


PEER_DATA_KERNELS = ("PushOp", "DirectOp", "OptOp")  # kernels whose stores peers read after a flag barrier


def test_system_scope_stores_are_waited_for_before_the_wave_ends(kernels):
    """the kernels that write data peers read (flag words — the barrier's own
    release store, a host-mapped error word — are polled, not published)"""
    ks = {k: v for k, v in kernels.items() if any(p in k for p in PEER_DATA_KERNELS)}
    assert ks
    bad = {k: b for k, v in ks.items() if (b := _unwaited(v))}
    assert not bad, "\n".join(f"{k}: {b[0]}" for k, b in list(bad.items())[:5])


def test_barrier_uses_system_scope_flags(kernels):
    """the flag barrier: system-scope release before the flag store (a
    write-back of this GPU's L2, `buffer_wbl2 sc0 sc1`) and acquire loads
    that bypass every cache level (sc0 sc1)"""
    ks = [v for k, v in kernels.items() if "xbarrier" in k]
    assert len(ks) == 1
    code = ks[0]
    assert any(i.startswith("buffer_wbl2") and "sc1" in i for i in code), "no system-scope release"
    assert any(i.startswith("global_load_dwordx2") and " sc0" in i and " sc1" in i for i in code), \
        "flag loads are not system coherent"


def test_checker_sees_a_missing_wait():
    """the checker itself: a sys store followed by s_endpgm with no wait fails"""
    assert _unwaited(["global_store_dwordx4 v[0:1], v[2:5], off sc0 sc1", "s_endpgm"])
    assert not _unwaited(["global_store_dwordx4 v[0:1], v[2:5], off sc0 sc1", "s_waitcnt vmcnt(0)", "s_endpgm"])
    assert _unwaited(["global_store_dword v0, v1, s[0:1] sc0 sc1", "s_cbranch_execz 3", "s_waitcnt vmcnt(0)"])


# ---- cache policy of the stream kernels (round 2: a run-time flag once let the
# compiler merge DirectOp's two load forms and drop the non-temporal hint)
def _vec_loads(code):
    return [i for i in code if i.startswith("global_load_dwordx")]


def _one_shot(kernels, op):
    """the one-shot (loop-free) instances of ew_kernel<op...>"""
    return {k: v for k, v in kernels.items()
            if "ew_kernel" in k and op in k and re.search(r"Lb0E(Li\d+E)?EEvT_mmm$", k)}


def test_direct_chain_reads_received_slices_non_temporal(kernels):
    """DirectOp<K, W, ZALL = false>: the K-1 received slices with nt loads, the
    owner's own slice (zeroed in the same pass) with a plain load"""
    ks = {k: v for k, v in _one_shot(kernels, "DirectOp").items() if re.search(r"DirectOpILi\d+E[tf]Lb0E", k)}
    assert ks
    for k, code in ks.items():
        m = re.search(r"DirectOpILi(\d+)E", k)
        K = int(m.group(1))
        loads = _vec_loads(code)
        nt = [i for i in loads if " nt" in i]
        assert len(loads) == K and len(nt) == K - 1, f"{k}: {len(nt)} nt of {len(loads)} vector loads"


def test_optimizer_and_sum_scale_stream_non_temporal(kernels):
    for op in ("OptOp", "SumScaleOp"):
        for k, code in _one_shot(kernels, op).items():
            if op == "SumScaleOp" and not re.search(r"SumScaleOpILi\d+ELi\dELb1E", k):
                continue  # the in-place form (out aliases an input) keeps plain loads
            loads = _vec_loads(code) + [i for i in code if i.startswith("global_load_lds_dwordx")]
            assert loads and all(" nt" in i for i in loads), f"{k}: {loads}"


def test_sum_scale_load_forms(kernels):
    """Round 3: K = 2 reads its inputs by LDS-DMA (two
    global_load_lds_dwordx4 nt, no VGPR loads); the serialized form for large
    buckets (SER, K >= 4) keeps ONE vector load in flight per wave: its K nt
    loads are each followed by vmcnt(0) before the next is issued; the
    small-bucket form keeps all K in flight."""
    ks = {k: v for k, v in _one_shot(kernels, "SumScaleOp").items() if re.search(r"SumScaleOpILi\d+ELi\dELb1E", k)}
    assert ks
    for k, code in ks.items():
        K = int(re.search(r"SumScaleOpILi(\d+)E", k).group(1))
        glds = [i for i in code if i.startswith("global_load_lds_dwordx4")]
        vec = [n for n, i in enumerate(code) if i.startswith("global_load_dwordx4")]
        if K == 2:
            assert len(glds) == 2 and not vec, f"{k}: {glds} {vec}"
        elif K >= 4:
            assert len(vec) == K and not glds, f"{k}: {len(vec)} vector loads"
            ser = re.search(r"SumScaleOpILi\d+ELi\dELb1ELb1E", k) is not None
            waits = [any(code[j] == "s_waitcnt vmcnt(0)" for j in range(a_ + 1, b_)) for a_, b_ in zip(vec, vec[1:])]
            assert all(waits) if ser else not any(waits), f"{k}: serialized={ser}, waits between loads {waits}"
    assert any(re.search(r"SumScaleOpILi8ELi\dELb1ELb1E", k) for k in ks), "no serialized K = 8 instance"


def _kernel_descriptors(tmp_path) -> dict:
    """kernel name -> its 64-byte kernel descriptor (the `<name>.kd` symbols of
    every gfx950 code object in the library), read with a minimal ELF64 parser."""
    import struct

    lib = tmp_path / "lib.so"
    shutil.copy(LIB, lib)
    subprocess.run([OBJDUMP, "--offloading", str(lib)], check=True, cwd=tmp_path, capture_output=True)
    out = {}
    for f in sorted(os.listdir(tmp_path)):
        if "amdgcn" not in f or "gfx950" not in f:
            continue
        data = (tmp_path / f).read_bytes()
        shoff, = struct.unpack_from("<Q", data, 0x28)
        shentsize, shnum = struct.unpack_from("<HH", data, 0x3A)
        secs = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
        for sh in secs:
            if sh[1] != 2:  # SHT_SYMTAB
                continue
            strtab = secs[sh[6]]
            for j in range(sh[5] // 24):
                name_off, info, other, shndx, value, size = struct.unpack_from("<IBBHQQ", data, sh[4] + j * 24)
                end = data.index(b"\0", strtab[4] + name_off)
                name = data[strtab[4] + name_off:end].decode()
                if name.endswith(".kd") and size == 64 and shndx < shnum:
                    sec = secs[shndx]
                    off = sec[4] + (value - sec[3])
                    out[name[:-3]] = data[off:off + 64]
    return out


def test_no_kernel_reads_the_dispatch_packet(tmp_path):
    """No kernel asks for the dispatch-packet pointer.  The compiler requests it
    when it moves a run-time-indexed private array to LDS (the flat work-item id
    is computed from the packet's workgroup sizes): the packet lives in the
    host-visible queue, and every wave's read of it cost the sparse lift's
    pattern kernels 25 us per launch (34 -> 9.6 us when the array went)."""
    kds = _kernel_descriptors(tmp_path)
    assert kds, "no kernel descriptors found"
    uses = [k for k, kd in kds.items() if int.from_bytes(kd[56:58], "little") & 0x2]
    assert not uses, f"kernels reading the dispatch packet: {uses[:5]}"
