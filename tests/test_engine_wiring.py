"""Every device pointer the decode kernels address is wired by the engine (CPU, source check).

The step kernels read their buffers from DecArgs / DecWeights / DecState (csrc/decoder.hpp); the
engine fills those structs (csrc/engine.hip).  A member the kernels use but the engine never sets
stays null on the GPU and faults the card -- round 4's first GPU run of the (since removed)
three-launch decode did exactly that (DecArgs::ah0 / ah1 added to the kernels, never allocated by
the engine), and the
host emulation (tools/emu) could not see it because its harness allocates the structs itself.
This test parses the structs and requires, for every pointer member, an assignment in the engine
(DecArgs: `a.<m> =`; DecState: allocated through `&e->ds.<m>`; DecWeights: `dw.<m>` set).  The
decode launcher also refuses null buffers at run time (launch_greedy_decode)."""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "rnnt-inference_amd", "csrc")


def _struct_pointers(src, name):
    body = re.search(r"struct %s \{(.*?)\n\};" % name, src, re.S).group(1)
    out = []
    for line in body.splitlines():
        code = line.split("//")[0]
        if "*" not in code:
            continue
        decl = code.strip().rstrip(";")
        # "const float* F", "int32_t *time, *added", "const uint16_t* wp[2]"
        for part in decl.split(","):
            m = re.search(r"\*\s*(\w+)\s*(\[\d+\])?\s*$", part)
            if m:
                out.append((m.group(1), m.group(2)))
    return out


def test_decode_structs_are_fully_wired_by_the_engine():
    hpp = open(os.path.join(CSRC, "decoder.hpp")).read()
    eng = open(os.path.join(CSRC, "engine.hip")).read()
    args = _struct_pointers(hpp, "DecArgs")
    names = {n for n, _ in args}
    assert {"F", "hc", "G", "res", "res_len"} <= names, names
    missing = [n for n, _ in args if not re.search(r"\ba\.%s\s*=" % n, eng)]
    assert not missing, f"DecArgs members never set in engine.hip: {missing}"
    state = _struct_pointers(hpp, "DecState")
    assert {"time", "list", "live", "count"} <= {n for n, _ in state}
    missing = [n for n, _ in state if not re.search(r"&e->ds\.%s\b" % n, eng)]
    assert not missing, f"DecState members never allocated in engine.hip: {missing}"
    weights = _struct_pointers(hpp, "DecWeights")
    missing = [n for n, arr in weights
               if not re.search(r"\bdw\.%s%s\s*=" % (n, r"\[[^\]]+\]" if arr else ""), eng)]
    assert not missing, f"DecWeights members never set in engine.hip: {missing}"


def test_launcher_refuses_null_buffers():
    src = open(os.path.join(CSRC, "decoder.hip")).read()
    body = src[src.index("int launch_greedy_decode("):]
    body = body[: body.index("\n}\n")]
    need = re.search(r"const void\* need\[\] = \{(.*?)\};", body, re.S).group(1)
    hpp = open(os.path.join(CSRC, "decoder.hpp")).read()
    for n, _ in _struct_pointers(hpp, "DecArgs"):
        assert re.search(r"\ba\.%s\b" % n, need), f"launch_greedy_decode does not check a.{n}"
