"""Client of the host-sanitizer driver (tests/native/host_rpc.cpp): the host-only
entry points of libpomcp_hip.so (csrc/host_api.cpp) compiled with
-fsanitize=address,undefined into an executable and called through the same
ctypes-style interface the product code uses, so tests/test_env_model.py and
tests/test_host_exp.py run them under the sanitizers unchanged
(tests/test_host_sanitize.py swaps this in for ``_native.load()``).  Any
sanitizer report aborts the driver; the next call then raises with its
report."""
import ctypes as C
import os
import shutil
import subprocess
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "tests", "native", "host_rpc.cpp"),
       os.path.join(ROOT, "posggym-baselines_amd", "csrc", "host_api.cpp")]
FLAGS = ["-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
         "-fno-omit-frame-pointer", "-Wall", "-Wno-unknown-pragmas"]


def build(out_dir=None):
    """Compile the driver (g++ with ASan + UBSan); returns its path."""
    cxx = shutil.which("g++")
    if cxx is None:
        raise RuntimeError("g++ not found")
    out_dir = out_dir or tempfile.mkdtemp(prefix="pomcp_host_asan_")
    exe = os.path.join(out_dir, "host_rpc")
    cmd = [cxx] + FLAGS + ["-I" + os.path.join(ROOT, "include")] + SRC + ["-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


class SanitizerError(RuntimeError):
    pass


class SanitizedHostLib:
    """The host entry points over the driver's pipe; anything else is taken
    from the product library (`fallback`)."""

    def __init__(self, exe, fallback=None):
        env = dict(os.environ, ASAN_OPTIONS="abort_on_error=0:halt_on_error=1:detect_leaks=1",
                   UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
        self._err = tempfile.TemporaryFile()
        self._p = subprocess.Popen([exe], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                   stderr=self._err, env=env)
        self._fallback = fallback
        self._grids = {}
        self.calls = 0

    # ----------------------------------------------------------- transport
    def _report(self):
        self._err.seek(0)
        return self._err.read().decode(errors="replace")[-4000:]

    def _call(self, line, payload=b""):
        self.calls += 1
        try:
            self._p.stdin.write(line.encode() + b"\n" + payload)
            self._p.stdin.flush()
            r = self._p.stdout.readline()
        except BrokenPipeError:
            r = b""
        if not r:
            self._p.wait(timeout=30)
            raise SanitizerError(f"host driver exited ({self._p.returncode}) on {line[:60]!r}:\n"
                                 + self._report())
        return [int(x) for x in r.split()]

    def _read(self, nbytes):
        buf = self._p.stdout.read(nbytes)
        if len(buf) != nbytes:
            raise SanitizerError("short read:\n" + self._report())
        return buf

    def _grid(self, kind, ref):
        raw = bytes(ref._obj)
        if self._grids.get(kind) != raw:
            assert self._call(f"{kind} {raw.hex()}") == [0]
            self._grids[kind] = raw

    def close(self):
        """Ends the driver; returns (exit status, its stderr)."""
        if self._p.poll() is None:
            try:
                self._p.stdin.write(b"quit\n")
                self._p.stdin.flush()
            except BrokenPipeError:
                pass
            self._p.wait(timeout=60)
        return self._p.returncode, self._report()

    def __getattr__(self, name):
        if self._fallback is None:
            raise AttributeError(name)
        return getattr(self._fallback, name)

    # ---------------------------------------------------- Driving-v1 (host)
    def pomcp_driving_sample_initial_state(self, g, seed, tree, ctr, out):
        self._grid("G", g)
        rc, c, s0, s1 = self._call(f"dsi {int(seed)} {int(tree)} {ctr._obj.value}")
        ctr._obj.value, out[0], out[1] = c, s0, s1
        return rc

    def pomcp_driving_obs(self, g, st, keys):
        self._grid("G", g)
        rc, k0, k1 = self._call(f"dobs {st[0]} {st[1]}")
        keys[0], keys[1] = k0, k1
        return rc

    def pomcp_driving_step(self, g, seed, tree, ctr, st, act, nxt, rew, term, keys):
        self._grid("G", g)
        v = self._call(f"dstep {int(seed)} {int(tree)} {ctr._obj.value} {st[0]} {st[1]} "
                       f"{act[0]} {act[1]}")
        ctr._obj.value = v[1]
        self._step_out(v, nxt, rew, term, keys)
        return v[0]

    @staticmethod
    def _step_out(v, nxt, rew, term, keys):
        nxt[0], nxt[1] = v[2], v[3]
        rew[0], rew[1] = (float(np.uint64(x).view(np.float64)) for x in v[4:6])
        term[0], term[1] = v[6], v[7]
        keys[0], keys[1] = v[8], v[9]

    # --------------------------------------------- PursuitEvasion-v1 (host)
    def pomcp_pe_sample_initial_state(self, g, seed, tree, ctr, out):
        self._grid("P", g)
        rc, c, s0, s1 = self._call(f"pesi {int(seed)} {int(tree)} {ctr._obj.value}")
        ctr._obj.value, out[0], out[1] = c, s0, s1
        return rc

    def pomcp_pe_obs(self, g, st, keys):
        self._grid("P", g)
        rc, k0, k1 = self._call(f"peobs {st[0]} {st[1]}")
        keys[0], keys[1] = k0, k1
        return rc

    def pomcp_pe_step(self, g, st, act, nxt, rew, term, keys):
        self._grid("P", g)
        v = self._call(f"pestep {st[0]} {st[1]} {act[0]} {act[1]}")
        self._step_out(v, nxt, rew, term, keys)
        return v[0]

    # ------------------------------------------------ RNG words / tables
    def pomcp_philox_words(self, seed, tree, stream, first, n, out):
        rc, m = self._call(f"philox {int(seed)} {int(tree)} {int(stream)} {int(first)} {int(n)}")
        words = np.frombuffer(self._read(4 * max(m, 0)), dtype=np.uint32)
        if m > 0:
            np.ctypeslib.as_array(C.cast(out, C.POINTER(C.c_uint32)), shape=(m,))[:] = words
        return rc

    def pomcp_host_log_table(self, first, n, out):
        rc, m = self._call(f"logtab {int(first)} {int(n)}")
        vals = np.frombuffer(self._read(8 * max(m, 0)), dtype=np.float64)
        if m > 0:
            np.ctypeslib.as_array(C.cast(out, C.POINTER(C.c_double)), shape=(m,))[:] = vals
        return rc

    def pomcp_debug_host_exp(self, x, n, out):
        n = int(n)
        xs = np.ctypeslib.as_array(C.cast(x, C.POINTER(C.c_double)), shape=(n,)).copy()
        rc, m = self._call(f"hexp {n}", xs.tobytes())
        vals = np.frombuffer(self._read(8 * m), dtype=np.float64)
        np.ctypeslib.as_array(C.cast(out, C.POINTER(C.c_double)), shape=(n,))[:] = vals
        return rc
