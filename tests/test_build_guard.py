"""The exec-narrowing build guard (cuda-raytracing_amd/build.py check_exec_narrowing) against saved
llvm-objdump text: the round-4 6-wave miscompile (tools/w6_repro.sh) must be found, the
same narrowing with an empty flow block must not, and a code object the parser cannot read must fail
the build instead of passing blind.  CPU only."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("rt_build", os.path.join(ROOT, "cuda-raytracing_amd", "build.py"))
build = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(build)

K = "_Z21render_fast_kernel_w6ILi30ELb0ELi21EEvPK15rt_render_args"


def _line(addr, text, enc="BF800000", target=None):
    tail = f" <{K}+0x{target:x}>" if target is not None else ""
    return f"\t{text:<58}// {addr:012X}: {enc}{tail}"


def _snippet(copy_behind_target):
    """The ISA shape of DESIGN.md 4.1's excerpt: cluster record loaded, exec narrowed without a save,
    execz branch to the join block, which holds (or not) the allocator's live-range copies before the
    parent's restore."""
    base = 0x1000
    rows = [f"{base:016x} <{K}>:"]
    a = base
    body = [
        ("s_and_saveexec_b64 s[14:15], vcc", None),
        ("global_load_dwordx4 v[60:63], v[2:3], off", None),
        ("s_waitcnt vmcnt(0)", None),
        ("v_cmp_lt_f32_e32 vcc, v60, v61", None),
        ("s_and_b64 exec, exec, vcc", None),
        ("s_cbranch_execz 4", "T"),
        ("v_max_f32_e32 v4, v60, v62", None),
        ("v_min_f32_e32 v5, v61, v63", None),
    ]
    addrs = []
    for text, tgt in body:
        addrs.append((a, text, tgt))
        a += 4 if not text.startswith("global") else 8
    target_addr = a
    join = ([("v_mov_b64 v[60:61], v[74:75]", None), ("v_mov_b64 v[62:63], v[76:77]", None)]
            if copy_behind_target else [])
    join += [("s_or_b64 exec, exec, s[14:15]", None), ("s_endpgm", None)]
    for text, tgt in join:
        addrs.append((a, text, tgt))
        a += 4
    for ad, text, tgt in addrs:
        rows.append(_line(ad, text, target=(target_addr - base) if tgt == "T" else None))
    return "\n".join(rows) + "\n"


def test_parser_reads_objdump_lines():
    base, ins = build.parse_disassembly(_snippet(True))
    assert base[K] == 0x1000
    assert len(ins) == 12
    br = [i for i in ins if i[1].startswith("s_cbranch_execz")]
    assert len(br) == 1 and br[0][2] == (K, 0x24)


def test_round4_hazard_is_found():
    hz = build.exec_narrowing_hazards(_snippet(True))
    assert len(hz) == 1
    k, addr, bad = hz[0]
    assert k == K and addr == 0x1014
    assert bad == ["v_mov_b64 v[60:61], v[74:75]", "v_mov_b64 v[62:63], v[76:77]"]


def test_empty_flow_block_is_clean():
    assert build.exec_narrowing_hazards(_snippet(False)) == []


def test_guard_raises_and_drops_flagged_objects(tmp_path, monkeypatch):
    bad, good = tmp_path / "bad.hip.o", tmp_path / "good.hip.o"
    for p in (bad, good):
        p.write_bytes(b"x")
        (tmp_path / (p.name + ".cmd")).write_text("cmd")
    texts = {str(bad): _snippet(True), str(good): _snippet(False)}
    monkeypatch.setattr(build, "disassemble", lambda o: texts[o])
    with pytest.raises(RuntimeError, match="without a save"):
        build.check_exec_narrowing([str(bad), str(good)])
    assert not bad.exists() and not (tmp_path / "bad.hip.o.cmd").exists()
    assert good.exists() and (tmp_path / "good.hip.o.cmd").exists()


def test_unparsable_device_code_fails(tmp_path, monkeypatch):
    obj = tmp_path / "odd.hip.o"
    obj.write_bytes(b"x")
    monkeypatch.setattr(build, "disassemble", lambda o: "some new objdump format\n\tv_mov_b32 v0, v1\n")
    with pytest.raises(RuntimeError, match="no instruction parsed"):
        build.check_exec_narrowing([str(obj)])
    monkeypatch.setattr(build, "disassemble", lambda o: "")  # no device code: nothing to check
    build.check_exec_narrowing([str(obj)])


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "cuda-raytracing_amd", "build", "rt_fast_prod.hip.o")),
                    reason="product objects not built")
def test_product_objects_parse_and_are_clean():
    obj = os.path.join(ROOT, "cuda-raytracing_amd", "build", "rt_fast_prod.hip.o")
    dis = build.disassemble(obj)
    assert len(build.parse_disassembly(dis)[1]) > 10000
    assert build.exec_narrowing_hazards(dis) == []
