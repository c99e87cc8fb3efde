#!/usr/bin/env python3
"""`make sanitize` driver: runs the host stages under AddressSanitizer +
UndefinedBehaviorSanitizer and ThreadSanitizer (SURVEY §5 "Race detection /
sanitizers"; CPU only -- GPU sanitizers are not available on the MI355X pool).

  1. ASan/UBSan rtx_scene_check (JSON loader host/json_min.hpp +
     host/scene_json.hpp, the scene compiler csrc/rt_scene.cpp, camera setup)
     over every committed scene and a seeded corpus of malformed files:
     truncations, byte flips, deleted/duplicated spans, type confusions,
     out-of-range indices and counts, non-finite and huge numbers, deep
     nesting, empty containers.  Each run must end with status 0 (valid) or 1
     (rejected with a message) and no sanitizer report.
  2. TSan rtx_scene_check --threads 8 over all scenes: concurrent loading and
     compilation of distinct scenes (rt_api.h "Threading").
  3. The kernel-source emulator (tests/native/rt_emulate.cpp: rt_path.h and
     rt_scene.cpp built for the host) under ASan/UBSan, driven by
     tests/test_emulator.py with libasan preloaded into the interpreter.
  4. The CLI's CPU backend (host/rtx_cpu.cpp, round 5) through
     host/rtx_cpu_check.cpp: its row pool under TSan (8 threads) and its
     per-path code under ASan/UBSan, every scene rendered twice and the two
     frames required equal bit for bit.

Writes a log (default profiles/r02_sanitize.log) and exits non-zero on any
finding.
"""
import argparse
import glob
import json
import os
import random
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "real-time-ray-tracing-engine_amd")
SAN_ENV = {
    "ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:exitcode=86:detect_stack_use_after_return=1",
    "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1:exitcode=87",
    "TSAN_OPTIONS": "halt_on_error=1:exitcode=88",
}


def mutations(text, rng, n):
    """Seeded malformed variants of one scene file."""
    out = []
    L = len(text)
    for k in range(n):
        op = k % 6
        if op == 0:  # truncation
            out.append(text[: rng.randrange(L)])
        elif op == 1:  # byte flips
            b = bytearray(text.encode())
            for _ in range(rng.randint(1, 8)):
                b[rng.randrange(len(b))] = rng.randrange(256)
            out.append(b.decode("latin-1"))
        elif op == 2:  # delete a span
            i = rng.randrange(L)
            out.append(text[:i] + text[i + rng.randint(1, 200):])
        elif op == 3:  # duplicate a span
            i = rng.randrange(L)
            j = min(L, i + rng.randint(1, 300))
            out.append(text[:j] + text[i:j] + text[j:])
        elif op == 4:  # replace a number with an extreme value
            import re
            nums = [m.span() for m in re.finditer(r"-?\d+(\.\d+)?([eE][-+]?\d+)?", text)]
            if nums:
                a, b = nums[rng.randrange(len(nums))]
                v = rng.choice(["1e308", "-1e308", "0", "-0", "1e-320", "2147483648", "-2147483649",
                                "99999999999999999999", "-1", "NaN", "Infinity", "1e999"])
                out.append(text[:a] + v + text[b:])
        else:  # replace a value with another JSON type
            import re
            ms = [m.span() for m in re.finditer(r":\s*(\[[^\[\]]*\]|\"[^\"]*\"|-?\d[\d.eE+-]*)", text)]
            if ms:
                a, b = ms[rng.randrange(len(ms))]
                v = rng.choice(['{}', '[]', '"x"', 'null', 'true', '[1,2]', '{"a":1}', '[[[]]]'])
                out.append(text[:a] + ": " + v + text[b:])
    return out


def handmade():
    """Structural edge cases the mutations rarely produce."""
    base = {"camera": {"image_width": 8}, "materials": {"m": {"type": "lambertian",
                                                              "albedo": [0.5, 0.5, 0.5]}}}
    cases = []

    def with_world(w, **extra):
        d = dict(base, world=w, **extra)
        return json.dumps(d)
    sphere = {"type": "sphere", "center": [0, 0, -1], "radius": 0.5, "material": "m"}
    cases.append("[" * 200000 + "]" * 200000)                    # deep nesting
    cases.append('{"a":' * 100000 + "1" + "}" * 100000)
    cases.append(with_world([]))                                  # empty world
    cases.append(with_world([sphere] * 3000))                     # many primitives
    cases.append(with_world([{"type": "list", "objects": []}]))
    nest = sphere
    for _ in range(64):                                           # deep transform chain
        nest = {"type": "translate", "offset": [0.01, 0, 0], "object": nest}
    cases.append(with_world([nest]))
    deep = ('{"type": "rotate_y", "angle": 1, "object": ' * 3000 + json.dumps(sphere)
            + "}" * 3000)
    cases.append(with_world(["@"]).replace('"@"', deep))
    cases.append(with_world([dict(sphere, material="nope")]))
    cases.append(with_world([dict(sphere, radius=-1)]))
    cases.append(with_world([dict(sphere, radius=float("inf"))]).replace("Infinity", "1e999"))
    cases.append(with_world([{"type": "quad", "Q": [0, 0, 0], "u": [0, 0, 0], "v": [0, 0, 0],
                              "material": "m"}]))             # degenerate quad
    cases.append(with_world([{"type": "medium", "density": 0.1, "boundary": sphere,
                              "albedo": [1, 1, 1]}]))
    cases.append(with_world([sphere], lights=[sphere] * 64))
    cases.append(with_world([sphere], camera={"image_width": 0}))
    cases.append(with_world([sphere], camera={"image_width": 100000, "aspect_ratio": 1e-9}))
    cases.append('{"camera": {"image_width": 8}, "world": [{"type": "sphere"}]}')
    cases.append('{"world": [{"type": "box", "a": [0,0,0], "b": [1,1,1]}]}')
    cases.append('"just a string"')
    cases.append("")
    cases.append("\x00\x01\x02")
    cases.append('{"world": "\\ud800\\u0000\\"\\\\"}')
    return cases


def run(cmd, env=None, timeout=600):
    e = dict(os.environ, **SAN_ENV)
    if env:
        e.update(env)
    return subprocess.run(cmd, capture_output=True, text=True, errors="replace", timeout=timeout,
                          env=e)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asan", required=True)
    ap.add_argument("--tsan", required=True)
    ap.add_argument("--emu-asan", default=None)
    ap.add_argument("--cpu-tsan", default=None)
    ap.add_argument("--cpu-asan", default=None)
    ap.add_argument("--only-cpu", action="store_true", help="run step 4 only")
    ap.add_argument("--log", default=os.path.join(ROOT, "profiles", "r02_sanitize.log"))
    ap.add_argument("--per-scene", type=int, default=150)
    a = ap.parse_args()
    log = []
    bad = 0
    scenes = sorted(glob.glob(os.path.join(PKG, "scenes", "*.json")))
    if a.only_cpu:
        bad += cpu_backend_steps(a, scenes, log)
        return finish(a, log, bad)

    # 1. valid scenes, ASan/UBSan
    r = run([a.asan] + scenes)
    log.append("[asan] committed scenes: rc %d\n%s%s" % (r.returncode, r.stdout, r.stderr))
    if r.returncode != 0:
        bad += 1

    # 1b. malformed corpus
    rng = random.Random(20261016)
    corpus = handmade()
    for p in scenes:
        corpus += mutations(open(p).read(), rng, a.per_scene)
    counts = {0: 0, 1: 0}
    with tempfile.TemporaryDirectory() as td:
        files = []
        for k, text in enumerate(corpus):
            f = os.path.join(td, "case%05d.json" % k)
            with open(f, "w", encoding="latin-1", errors="replace") as fh:
                fh.write(text)
            files.append(f)
        for k in range(0, len(files), 50):  # batches keep the sanitizer start-up cost low
            batch = files[k:k + 50]
            r = run([a.asan] + batch)
            if r.returncode not in (0, 1) or "Sanitizer" in r.stderr or "runtime error" in r.stderr:
                # isolate the offending file(s)
                for f in batch:
                    r1 = run([a.asan, f])
                    if r1.returncode not in (0, 1) or "Sanitizer" in r1.stderr or \
                            "runtime error" in r1.stderr:
                        bad += 1
                        log.append("[asan] FINDING on %s (rc %d):\n%s\n--- input head: %r" % (
                            os.path.basename(f), r1.returncode, r1.stderr[-4000:],
                            open(f, encoding="latin-1").read()[:300]))
                    else:
                        counts[r1.returncode] += 1
            else:
                for line in r.stdout.splitlines():
                    counts[0 if line.split(": ", 1)[1].startswith("ok") else 1] += 1
    log.append("[asan] malformed corpus: %d files, %d accepted, %d rejected cleanly, %d findings" % (
        len(corpus), counts[0], counts[1], bad))

    # 2. TSan, concurrent compilation of distinct scenes
    r = run([a.tsan, "--threads", "8", "--repeat", "3"] + scenes)
    log.append("[tsan] 8 threads x 3 repeats over %d scenes: rc %d\n%s%s" % (
        len(scenes), r.returncode, r.stdout, r.stderr[-4000:]))
    if r.returncode != 0:
        bad += 1

    # 3. emulator under ASan/UBSan through its pytest driver
    if a.emu_asan:
        libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True,
                                 text=True).stdout.strip()
        env = {"LD_PRELOAD": libasan, "RTX_EMU_LIB": a.emu_asan,
               "ASAN_OPTIONS": "detect_leaks=0:exitcode=86"}
        r = run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                 os.path.join(ROOT, "tests", "test_emulator.py")], env=env, timeout=1800)
        tail = "\n".join(r.stdout.strip().splitlines()[-3:])
        log.append("[asan] kernel-source emulator (tests/test_emulator.py): rc %d\n%s\n%s" % (
            r.returncode, tail, r.stderr[-3000:] if r.returncode else ""))
        if r.returncode != 0:
            bad += 1

    bad += cpu_backend_steps(a, scenes, log)
    finish(a, log, bad)


def cpu_backend_steps(a, scenes, log):
    """4. the CPU backend: TSan over its row pool, ASan/UBSan over the path code."""
    bad = 0
    for tag, exe, threads in (("tsan", a.cpu_tsan, 8), ("asan", a.cpu_asan, 4)):
        if not exe:
            continue
        r = run([exe, "--threads", str(threads)] + scenes, timeout=1800)
        log.append("[%s] CPU backend (host/rtx_cpu_check.cpp), %d threads over %d scenes: rc %d\n%s%s" % (
            tag, threads, len(scenes), r.returncode, r.stdout, r.stderr[-4000:]))
        if r.returncode != 0 or "Sanitizer" in r.stderr or "runtime error" in r.stderr:
            bad += 1
    return bad


def finish(a, log, bad):
    log.append("RESULT: %s" % ("clean" if bad == 0 else "%d finding(s)" % bad))
    os.makedirs(os.path.dirname(a.log), exist_ok=True)
    with open(a.log, "w") as f:
        f.write("\n\n".join(log) + "\n")
    print("\n".join(x.splitlines()[0] for x in log))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
