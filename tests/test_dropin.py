"""The drop-in boundary at the source level: the reference's own CLI driver,
/root/reference/src/llama.cpp, compiles UNCHANGED against include/ and links to libthallama.so
in place of its thaBLAS/thaDNN/models sources (oracle/Makefile `_ref/llama_on_thallama`).

CPU: the compile + link (only where /root/reference exists), the headers' reference signatures
(C++ references for the out-parameters, reference include/models.hpp:120-134) and their C view.
GPU: that binary — the reference's scheduler, tokenizer and sampler driving our library — writes
the same `-m test` output file as the CPU restatement of the reference (tests/test_cli_gpu.py)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
INC = os.path.join(REPO, "include")
LIBDIR = os.path.join(REPO, "hip_llama.cpp_amd", "lib")
BUILT = os.path.join(REPO, "oracle", "_ref", "llama_on_thallama")
HIPCC = "/opt/rocm/bin/hipcc"
need_ref = pytest.mark.skipif(not os.path.exists(os.path.join(REF, "src", "llama.cpp")),
                              reason="the reference tree is not on this machine")


@need_ref
def test_reference_cli_compiles_and_links_unchanged(tmp_path):
    exe = tmp_path / "llama"
    r = subprocess.run([HIPCC, "-O1", "-std=c++17", "-fopenmp", "--offload-arch=gfx950", "-I" + INC, "-o", str(exe),
                        os.path.join(REF, "src", "llama.cpp"), os.path.join(REF, "src", "seq.cpp"),
                        os.path.join(REF, "src", "utils.cpp"), "-L" + LIBDIR, "-lthallama",
                        "-Wl,-rpath," + LIBDIR], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    # every thaBLAS / thaDNN / device-residency symbol it uses comes from libthallama.so
    und = subprocess.run(["nm", "-u", str(exe)], capture_output=True, text=True, check=True).stdout
    for name in ["thablasCreate", "thaDNN_s_forward_batch", "copy_weight_to_device", "alloc_state_to_device_batch",
                 "thaDNN_s_forward_70B", "alloc_state_to_device_70B",
                 "thaDNN_s_forward_batch_multiple_pipe_line_layer_swap"]:
        assert f" U {name}\n" in und, name
    ldd = subprocess.run(["ldd", str(exe)], capture_output=True, text=True).stdout
    assert "libthallama.so" in ldd
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert run.returncode != 0 and "Usage:" in run.stderr  # its own argument parsing (src/llama.cpp:1489-1505)


CXX_SIGNATURES = r"""
#include "seq.hpp"
#include "thaDNN.hpp"
#include "thaBLAS.hpp"
#include "utils.hpp"
#include <type_traits>
// reference include/models.hpp:120-134 and include/thaDNN.hpp:69-80, exactly
static_assert(std::is_same<decltype(&copy_weight_to_device), void (*)(Transformer*, TransformerWeights*&)>::value, "");
static_assert(std::is_same<decltype(&alloc_state_to_device_batch), void (*)(Transformer*, RunState*&, int)>::value, "");
static_assert(std::is_same<decltype(&alloc_state_to_device), void (*)(Transformer*, RunState*&)>::value, "");
static_assert(std::is_same<decltype(&copy_transformer_to_device),
                           void (*)(thablasHandle_t, Transformer*, Transformer*&)>::value, "");
static_assert(std::is_same<decltype(&alloc_state_to_device_70B), void (*)(Transformer*, RunState*&)>::value, "");
static_assert(std::is_same<decltype(&alloc_weight_to_device_70B), void (*)(Transformer*, TransformerWeights*&)>::value, "");
static_assert(std::is_same<decltype(&copy_transformer_weight_pipeline_to_device_batch),
                           void (*)(Transformer*, TransformerWeights*&, int, int, int)>::value, "");
static_assert(std::is_same<decltype(&thaDNN_s_forward_batch),
                           thablasStatus_t (*)(thablasHandle_t, thablasHandle_t, thablasHandle_t, int, Config*,
                                               TransformerWeights*, RunState*, int*, int*, float*)>::value, "");
static_assert(std::is_same<decltype(&thaDNN_s_forward_70B),
                           thablasStatus_t (*)(thablasHandle_t, int, Config*, TransformerWeights**, RunState*,
                                               TransformerWeights*, RunState*, int*, int*, float*)>::value, "");
static_assert(sizeof(Config) == 28 && sizeof(TransformerWeights) == 12 * sizeof(void*) &&
              sizeof(RunState) == 16 * sizeof(void*), "reference layouts");
int main() { return 0; }
"""

C_VIEW = r"""
#include "thallama.h"
#include "thaDNN.hpp"
/* the same symbols seen from C: out-parameters are pointers to the pointers */
static void (*f1)(Transformer*, TransformerWeights**) = copy_weight_to_device;
static void (*f2)(Transformer*, RunState**, int) = alloc_state_to_device_batch;
int main(void) { return f1 == 0 || f2 == 0; }
"""


def test_header_signatures_match_the_reference(tmp_path):
    src = tmp_path / "sig.cpp"
    src.write_text(CXX_SIGNATURES)
    r = subprocess.run([HIPCC, "-std=c++17", "-fsyntax-only", "-I" + INC, str(src)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]


def test_headers_have_a_c_view(tmp_path):
    src = tmp_path / "view.c"
    src.write_text(C_VIEW)
    r = subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-x", "c", "-I" + INC, "-I/opt/rocm/include",
                        "-D__HIP_PLATFORM_AMD__", str(src)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]


def test_reference_artefact_name_built():
    """The CLI also ships under the reference's artefact path (reference Makefile:5-7)."""
    exe = os.path.join(REPO, "build", "apps", "llama")
    assert os.path.exists(exe), "make -C hip_llama.cpp_amd"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "Usage:" in r.stderr
    assert os.path.exists(os.path.join(REPO, "assets", "tokenizer.bin"))  # its default -z (src/llama.cpp:1520)


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 3, 9])
def test_reference_cli_on_the_library_test_mode(gpu, oracle, pkg, tmp_path, batch):
    """The reference's UNCHANGED src/llama.cpp (built by oracle/Makefile against libthallama.so)
    writes the byte-identical `-m test` output file that the CPU restatement of the reference
    produces (its scheduler with `batch` slots; 9 > 7 prompts leaves slots that never get a
    request, whose token/pos the reference leaves uninitialised)."""
    if not os.path.exists(BUILT):
        pytest.skip("oracle/_ref/llama_on_thallama not built (needs the reference tree at build time)")
    import test_cli_gpu as T
    from hip_llama_cpp_amd import host as H
    base = oracle.Model(T.CFG, 0, seed=2024)
    arena = base.arena().copy()
    arena[-T.V * T.CFG[0]:] *= 30.0
    ref = oracle.Model(T.CFG, 0, payload=arena)
    path = str(tmp_path / "model.bin")
    ref.write_v0(path)
    inp = tmp_path / "in.txt"
    inp.write_bytes((f"{len(T.PROMPTS)}\n" + "\n".join(T.PROMPTS) + "\n").encode())
    out = tmp_path / "out.txt"
    shutil.copy(T.TOK, tmp_path / "tokenizer.bin")
    r = subprocess.run([BUILT, path, "-m", "test", "-f", str(inp), "-o", str(out), "-b", str(batch), "-z",
                        str(tmp_path / "tokenizer.bin")], cwd=tmp_path, capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    want, _ = T.expected_test_mode(H, ref, T.PROMPTS, T.CFG[6])
    assert out.read_bytes() == f"{len(T.PROMPTS)}\n".encode() + b"".join(w + b"\n" for w in want)


@pytest.mark.gpu
def test_reference_cli_timed_beside_ours(gpu, oracle, pkg, tmp_path):
    """The drop-in's cost as the reference's own driver uses it: its UNCHANGED src/llama.cpp test
    mode on libthallama.so — per step an H2D of token/pos, thaDNN_s_forward_batch, a D2H of the
    B x V logits, a device synchronisation and host sampling (src/thaDNN.cpp:24-79,
    src/llama.cpp:1024-1050) — timed beside this repository's CLI (build/apps/llama, the same
    sampling) on the same stories110M-shaped v0 file and the first 16 prompts of the reference's
    gen_in_128.txt, each request to seq_len 1024 or BOS/EOS, 8 slots.  The classifier is scaled
    (peaked distributions) so both samplers draw the same tokens from logits within 1e-4: the two
    output files must be equal.  Both throughputs (the reference's own "achieved throughput" line)
    go to gpurun_out/dropin_timing.json."""
    import json
    import time
    if not os.path.exists(BUILT):
        pytest.skip("oracle/_ref/llama_on_thallama not built (needs the reference tree at build time)")
    cfg = (768, 2048, 12, 12, 12, 32000, 1024)
    base = oracle.Model(cfg, 0, seed=110)
    arena = base.arena().copy()
    arena[-cfg[5] * cfg[0]:] *= 30.0
    path = str(tmp_path / "stories110m_peaked.bin")
    oracle.Model(cfg, 0, payload=arena).write_v0(path)
    with open(os.path.join(REPO, "tests", "golden", "gen_in_128.txt"), "rb") as f:
        lines = f.read().split(b"\n")
    n = 16
    inp = tmp_path / "in.txt"
    inp.write_bytes(f"{n}\n".encode() + b"\n".join(lines[1:1 + n]) + b"\n")
    shutil.copy(os.path.join(REPO, "tests", "golden", "tokenizer.bin"), tmp_path / "tokenizer.bin")
    res = {}
    outs = {}
    ours = os.path.join(REPO, "build", "apps", "llama")
    for name, exe, env in (("reference_cli_on_libthallama", BUILT, {}), ("this_cli", ours, {}),
                           ("this_cli_prompts_stepped", ours, {"THALLAMA_NO_PREFILL": "1"})):
        out = tmp_path / f"out_{name}.txt"
        t0 = time.perf_counter()
        r = subprocess.run([exe, path, "-m", "test", "-f", str(inp), "-o", str(out), "-b", "8", "-z",
                            str(tmp_path / "tokenizer.bin")], cwd=tmp_path, capture_output=True, text=True, timeout=600,
                           env={**os.environ, **env})
        wall = time.perf_counter() - t0
        assert r.returncode == 0, r.stderr[-2000:]
        tot = [ln for ln in r.stdout.splitlines() if ln.startswith("Total achieved token:")]
        el = [ln for ln in r.stdout.splitlines() if ln.startswith("elapsed time(s):")]
        tokens, secs = int(tot[-1].split()[-1]), float(el[-1].split()[2].rstrip(","))
        res[name] = {"tokens": tokens, "seconds": secs, "tok_s": round(tokens / secs, 1), "wall_s": round(wall, 2)}
        outs[name] = out.read_bytes()
    res["outputs_equal"] = outs["reference_cli_on_libthallama"] == outs["this_cli"] == outs["this_cli_prompts_stepped"]
    res["workload"] = (f"stories110M-shaped fp32 v0 file (classifier x30), first {n} prompts of gen_in_128.txt, -m test "
                       "-b 8 (T=1.0, top-p 0.9, seed 314028 per request), each request to seq_len 1024 or BOS/EOS")
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "dropin_timing.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    assert res["outputs_equal"]
    assert res["reference_cli_on_libthallama"]["tokens"] == res["this_cli"]["tokens"]


@pytest.mark.gpu
@pytest.mark.slow
def test_reference_cli_timed_beside_ours_7b(gpu, oracle, pkg, tmp_path):
    """The drop-in contract priced at the size config[4] multiplies: the reference's UNCHANGED
    src/llama.cpp test mode on libthallama.so at 8 slots on a llama2-7B-shaped v0 file — per step an
    H2D of token/pos, thaDNN_s_forward_batch, a D2H of the 8 x 32000 logits, hipDeviceSynchronize and
    host sampling (src/thaDNN.cpp:24-79, src/llama.cpp:1017-1050) — beside this repository's CLI in
    the same mode (host sampling, prompts stepped like the reference: THALLAMA_NO_PREFILL=1) and with
    its prefill, on the first 8 prompts of gen_in_64.txt.  The file's header says seq_len 256, so
    each request runs to position 255 or BOS/EOS (the reference's test mode always runs to seq_len).
    Same library, same decoder, same sampler: the reference's file and ours with prompts stepped
    must be byte-identical.  Throughputs go to gpurun_out/dropin_timing_7b.json."""
    import json
    import time
    if not os.path.exists(BUILT):
        pytest.skip("oracle/_ref/llama_on_thallama not built (needs the reference tree at build time)")
    if shutil.disk_usage(str(tmp_path)).free < 40 * 2**30:
        pytest.skip("less than 40 GiB free for the 27 GB model file")
    cfg = (4096, 11008, 32, 32, 32, 32000, 256)
    path = str(tmp_path / "llama2_7b_synth_s256.bin")
    oracle.set_threads(min(16, os.cpu_count() or 1))
    t0 = time.perf_counter()
    m = oracle.Model(cfg, 0, seed=20240224)
    m.write_v0(path)
    m.close()
    del m
    made_s = time.perf_counter() - t0
    with open(os.path.join(REPO, "tests", "golden", "gen_in_64.txt"), "rb") as f:
        lines = f.read().split(b"\n")
    n = 8
    inp = tmp_path / "in.txt"
    inp.write_bytes(f"{n}\n".encode() + b"\n".join(lines[1:1 + n]) + b"\n")
    shutil.copy(os.path.join(REPO, "tests", "golden", "tokenizer.bin"), tmp_path / "tokenizer.bin")
    res, outs = {}, {}
    ours = os.path.join(REPO, "build", "apps", "llama")
    for name, exe, env in (("reference_cli_on_libthallama", BUILT, {}),
                           ("this_cli_prompts_stepped", ours, {"THALLAMA_NO_PREFILL": "1"}),
                           ("this_cli", ours, {})):
        out = tmp_path / f"out_{name}.txt"
        t1 = time.perf_counter()
        r = subprocess.run([exe, path, "-m", "test", "-f", str(inp), "-o", str(out), "-b", "8", "-z",
                            str(tmp_path / "tokenizer.bin")], cwd=tmp_path, capture_output=True, text=True, timeout=600,
                           env={**os.environ, **env})
        wall = time.perf_counter() - t1
        assert r.returncode == 0, r.stderr[-2000:]
        tot = [ln for ln in r.stdout.splitlines() if ln.startswith("Total achieved token:")]
        el = [ln for ln in r.stdout.splitlines() if ln.startswith("elapsed time(s):")]
        tokens, secs = int(tot[-1].split()[-1]), float(el[-1].split()[2].rstrip(","))
        res[name] = {"tokens": tokens, "seconds": secs, "tok_s": round(tokens / secs, 1), "wall_s": round(wall, 2)}
        outs[name] = out.read_bytes()
        print(name, res[name], flush=True)
    res["files_equal_reference_vs_stepped"] = outs["reference_cli_on_libthallama"] == outs["this_cli_prompts_stepped"]
    res["workload"] = (f"llama2-7B-shaped fp32 v0 file (synthetic, seed 20240224, header seq_len 256), first {n} prompts "
                       "of gen_in_64.txt, -m test -b 8 (T=1.0, top-p 0.9, the reference's per-request seed), each "
                       "request to position 255 or BOS/EOS")
    res["model_file_s"] = round(made_s, 1)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "dropin_timing_7b.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    os.remove(path)
    assert res["files_equal_reference_vs_stepped"]
    assert res["reference_cli_on_libthallama"]["tokens"] == res["this_cli_prompts_stepped"]["tokens"]
