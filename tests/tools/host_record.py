#!/usr/bin/env python3
"""Record the host-only native calls of the query path (test infrastructure): every
mh_terms_create / mh_terms_set_options / mh_terms_append / mh_query_build / mh_terms_destroy,
mh_harvester_create /
mh_guide_harvest_with / mh_guide_harvest / mh_harvester_destroy and mh_smtlib_create / read /
commit / rollback / destroy the Python side makes, with the bytes of their arguments (and the
read's return code), into a file that tests/native/host_replay.cpp replays against a build of
csrc/query.cpp + harvest.cpp + smtlib.cpp under AddressSanitizer / UBSan
(tests/test_host_sanitized.py).

The workload is the query path's host half without a device: the LASER-shaped queries of
tests/laser_like.py and tests/laser_paths.py in LASER order (each prefix a query, svm.py:257-262),
their UNSAT variants, random conjunctions (tests/test_query_native._random_query) in LASER, BFS
and JUMPI order, and planted random paths with keccak applications as read columns, each
compiled by the native query compiler and, when not refuted, harvested by a guide session; and
the z3-printed text of every LASER-shaped query read constraint by constraint into one SMT-LIB
session (tests/z3_style.py), plus malformed texts the reader must refuse.

    python tests/tools/host_record.py OUT [n_random]
"""
import ctypes as C
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)

from mythril_amd import native  # noqa: E402

NODE = native.NODE_DTYPE.itemsize


def _bytes(p, n):
    if n == 0:
        return b""
    addr = p if isinstance(p, int) else C.cast(p, C.c_void_p).value
    return C.string_at(addr, n)


class Recorder:
    """Stands in for the loaded CDLL: the recorded entry points write a record and forward."""

    def __init__(self, lib, out):
        self.lib, self.out = lib, out

    def __getattr__(self, name):
        return getattr(self.lib, name)

    def _w(self, kind, sid, payload=b""):
        self.out.write(struct.pack("<cQQ", kind, sid, len(payload)) + payload)

    @staticmethod
    def _handle(pp):
        return pp._obj.value or 0

    def mh_terms_create(self, pp):
        r = self.lib.mh_terms_create(pp)
        self._w(b"C", self._handle(pp))
        return r

    def mh_terms_set_options(self, h, options):
        self._w(b"O", h.value or 0, struct.pack("<I", options))
        return self.lib.mh_terms_set_options(h, options)

    def mh_terms_destroy(self, h):
        self._w(b"D", h.value or 0)
        return self.lib.mh_terms_destroy(h)

    def mh_terms_append(self, h, nodes, n_nodes, consts, n_consts, vn, n_vars, an, n_arrays,
                        fn, n_fns):
        p = struct.pack("<Q", n_nodes) + _bytes(nodes, n_nodes * NODE)
        p += struct.pack("<Q", n_consts) + _bytes(consts, n_consts * 32)
        for names, n in ((vn, n_vars), (an, n_arrays), (fn, n_fns)):
            p += struct.pack("<QQ", n, len(names)) + names
        self._w(b"A", h.value or 0, p)
        return self.lib.mh_terms_append(h, nodes, n_nodes, consts, n_consts, vn, n_vars, an,
                                        n_arrays, fn, n_fns)

    def mh_query_build(self, h, roots, n_roots, out, info):
        self._w(b"Q", h.value or 0, struct.pack("<I", n_roots) + _bytes(roots, 4 * n_roots))
        return self.lib.mh_query_build(h, roots, n_roots, out, info)

    def mh_harvester_create(self, pp):
        r = self.lib.mh_harvester_create(pp)
        self._w(b"H", self._handle(pp))
        return r

    def mh_harvester_destroy(self, h):
        self._w(b"X", h.value or 0)
        return self.lib.mh_harvester_destroy(h)

    def _guide(self, kind, sid, args):
        nodes, n, consts, nc, widths, ncol, pc, pv, npar = args[:9]
        p = struct.pack("<I", n) + _bytes(nodes, n * NODE)
        p += struct.pack("<I", nc) + _bytes(consts, nc * 32)
        p += struct.pack("<I", ncol) + _bytes(widths, 2 * ncol)
        p += struct.pack("<I", npar) + _bytes(pc, 4 * npar) + _bytes(pv, 32 * npar)
        self._w(kind, sid, p)

    def mh_guide_harvest_with(self, s, *args):
        self._guide(b"G", s.value or 0, args)
        return self.lib.mh_guide_harvest_with(s, *args)

    def mh_guide_harvest_inc(self, *args):
        self._guide(b"i", 0, args)
        return self.lib.mh_guide_harvest_inc(*args)

    def mh_guide_harvest(self, *args):
        self._guide(b"g", 0, args)
        return self.lib.mh_guide_harvest(*args)

    def mh_smtlib_create(self, pp):
        r = self.lib.mh_smtlib_create(pp)
        self._w(b"S", self._handle(pp))
        return r

    def mh_smtlib_destroy(self, h):
        self._w(b"Z", h.value or 0)
        return self.lib.mh_smtlib_destroy(h)

    def mh_smtlib_read(self, h, data, n, batch):
        r = self.lib.mh_smtlib_read(h, data, n, batch)
        self._w(b"R", h.value or 0, struct.pack("<i", r) + bytes(data[:n]))
        return r

    def mh_smtlib_commit(self, h, ids, n):
        self._w(b"M", h.value or 0, struct.pack("<Q", n) + _bytes(ids, 8 * n))
        return self.lib.mh_smtlib_commit(h, ids, n)

    def mh_smtlib_rollback(self, h):
        self._w(b"B", h.value or 0)
        return self.lib.mh_smtlib_rollback(h)


def host_query(b, roots, guides, rng, keccak_reads=False):
    """The host half of Sieve.solve for one query: native compile, then the guide harvest."""
    cq = native.TermMirror.of(b, keccak_reads).build(b, roots)
    if cq.flags & (native.QUERY_REFUTED | native.QUERY_DEFINITIONS):
        return
    parent = []
    if len(cq.names) and rng.random() < 0.5:  # a parent witness for some columns
        parent = [(c, rng.getrandbits(256)) for c in rng.sample(range(len(cq.names)),
                                                                 min(3, len(cq.names)))]
    native.harvest_guide(cq.tapes[0], cq.consts, cq.widths, parent,
                         session=guides if rng.random() < 0.8 else None)


def workload(n_random=40):
    from tests.laser_like import hard_queries, queries
    from tests.laser_paths import grow
    from tests.test_query_native import _random_query

    rng = random.Random(1234)
    guides = native.GuideSession()

    def laser_order(b, nodes):
        for k in range(1, len(nodes) + 1):  # every prefix, parents first
            host_query(b, nodes[:k], guides, rng)

    def done(b):  # the builder's sessions end inside the recording
        for attr in ("_term_mirror", "_term_mirror_kr"):
            m = b.__dict__.pop(attr, None)
            if m is not None:
                m.close()

    for make in (queries, hard_queries):
        ctx, qs = make()
        for _, cs in qs:
            laser_order(ctx.b, [c.node for c in cs])
        done(ctx.b)
    for shape in ("killbilly", "overflow", "ether_thief"):
        for unsat in (False, True):
            ctx, cs = grow(shape, 60, unsat=unsat)
            laser_order(ctx.b, [c.node for c in cs])
            done(ctx.b)
    for seed in range(n_random):
        ctx, cs = _random_query(random.Random(seed), 3 + seed % 9)
        laser_order(ctx.b, [c.node for c in cs])
        done(ctx.b)
    # BFS order with both branches of every JUMPI (the query compiler's rollback and replay,
    # the harvester session's prefix truncation; tests/bfs_order.py)
    from mythril_amd.smt import Not
    from tests.bfs_order import bfs_queries

    for shape, k in (("killbilly", 4), ("ether_thief", 8), ("overflow", 4)):
        ctx, cs = grow(shape, 40)
        nodes, negs = [c.node for c in cs], [Not(c).node for c in cs]
        for roots in bfs_queries(nodes, negs, 20, k, k):
            host_query(ctx.b, roots, guides, rng)
        done(ctx.b)
    for seed in range(min(n_random, 12)):
        ctx, cs = _random_query(random.Random(500 + seed), 8)
        cs = [c for c in cs if hasattr(c, "node")]
        for roots in bfs_queries([c.node for c in cs], [Not(c).node for c in cs], 2, 4, seed):
            try:
                host_query(ctx.b, roots, guides, rng)
            except native.Unsupported:
                pass
        done(ctx.b)
    # the keccak second chance (MH_TERMS_KECCAK_READS): planted random paths in LASER order and
    # the random conjunctions in JUMPI order, on a session of that mode beside the default one
    from tests.planted import planted_path

    from mythril_amd.sieve import newest_tape

    for seed in range(min(n_random, 8)):
        ctx, cs, m, _ = planted_path("random", seed, 12)
        nodes = [c.node for c in cs]
        for k in range(1, len(nodes) + 1):
            host_query(ctx.b, nodes[:k], guides, rng)
            host_query(ctx.b, nodes[:k], guides, rng, keccak_reads=True)
            # the incremental round's guide: the newest root's conjuncts, the planted model's
            # values as the parent (mh_guide_harvest_inc)
            cq = native.TermMirror.of(ctx.b).build(ctx.b, nodes[:k])
            inc = newest_tape(cq.tapes[0], cq.parent_len) if cq.parent_len else None
            if inc is not None:
                par = [(i, m.vars[c]) for i, c in enumerate(cq.names) if c in m.vars]
                native.harvest_guide(inc, cq.consts, cq.widths, par, parent_eval=True)
        done(ctx.b)
    for seed in range(min(n_random, 8)):
        ctx, cs = _random_query(random.Random(900 + seed), 8)
        cs = [c for c in cs if hasattr(c, "node")]
        for k in range(1, len(cs) + 1):
            for roots in ([c.node for c in cs[:k]],
                          [c.node for c in cs[:k - 1]] + [Not(cs[k - 1]).node]):
                try:
                    host_query(ctx.b, roots, guides, rng, keccak_reads=True)
                except native.Unsupported:
                    pass
        done(ctx.b)
    guides.close()
    smtlib_workload()


def smtlib_workload():
    from mythril_amd import smtlib
    from tests.laser_like import hard_queries, queries
    from tests.z3_style import z3_sexpr

    nat = smtlib.NativeReader()
    for make in (queries, hard_queries):
        _, qs = make()
        for _, cs in qs:
            for c in cs:  # LASER order: one new constraint at a time, into one session
                nat.read(z3_sexpr(c), smtlib.Query(nat.ctx))
    for bad in ("(assert (bvadd #x01 #x0001))", "(assert (= y #x01))", "(assert (and true",
                "(declare-fun f ((_ BitVec 8) (_ BitVec 8)) (_ BitVec 8))", "(assert #x01)",
                "(assert (= ((_ extract 300 0) #x01) #x01))", ")", "(assert (let ((a!1 #x01))"):
        try:
            nat.read(bad, smtlib.Query(nat.ctx))
        except smtlib.SmtlibError:
            pass
    nat.session.close()


def main():
    out_path = sys.argv[1]
    n_random = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    real = native.load()
    with open(out_path, "wb") as f:
        native._lib = Recorder(real, f)
        try:
            workload(n_random)
        finally:
            native._lib = real


if __name__ == "__main__":
    main()
