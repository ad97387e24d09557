"""Multi-PE check of team management against SOS's rules (one process per PE).

Run under tools/oshrun.  Covers src/shmem_team.c:290-505 and src/teams_c.c4:
  * split_strided argument rules: stride 0 and 1-PE teams take stride 1, bad
    <start, stride, size> triplets return -1 on every PE without a collective;
  * the team-slot pool: SHMEM_TEAMS_MAX (default 10) minus WORLD/SHARED/NODE teams can
    exist at once; one more split returns 1 on every parent PE; destroy frees a slot;
  * split_2d: x teams are consecutive runs of xrange parent PEs, y teams stride xrange,
    checked through shmem_team_my_pe / n_pes / translate_pe and a sum reduction over
    each axis team (sum of world PE ids);
  * get_config / translate_pe / SHMEMX_TEAM_NODE.
Prints one line per PE, exit 0 = OK.
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from sos_amd import shmem as S  # noqa: E402

NUM_CONTEXTS = 1


class Config(ctypes.Structure):
    _fields_ = [("num_contexts", ctypes.c_int)]


def main():
    S.shmem_init()
    L = S.lib()
    me, P = S.shmem_my_pe(), S.shmem_n_pes()
    world = S.team_world()
    bad, checks = [], 0

    def check(ok, what):
        nonlocal checks
        checks += 1
        if not ok:
            bad.append(what)

    def split(parent, start, stride, size, cfg=None, mask=0):
        t = ctypes.c_void_p(0)
        rc = L.shmem_team_split_strided(parent, start, stride, size,
                                        ctypes.byref(cfg) if cfg is not None else None, mask,
                                        ctypes.byref(t))
        return rc, t.value

    def team_sum(team, members):
        """shmem_long_sum_reduce of the world PE id over `team` (host buffers)."""
        src = np.array([me], dtype=np.int64)
        dst = np.zeros(1, dtype=np.int64)
        S.shmem_long_sum_reduce(team, dst.ctypes.data, src.ctypes.data, 1)
        return int(dst[0]) == sum(members)

    # predefined teams
    node = S.team_node()
    check(node is not None and L.shmem_team_n_pes(node) == P and L.shmem_team_my_pe(node) == me,
          "node team")
    check(L.shmem_team_translate_pe(world, me, node) == me, "translate world->node")

    # argument rules: every PE sees -1, no collective is started
    for args in ((P, 1, 1), (0, 1, P + 1), (0, 1, 0), (-1, 1, 1), (0, 2, P) if P > 1 else (0, 1, 2)):
        rc, t = split(world, *args)
        check(rc == -1 and not t, ("bad triplet", args, rc))
    # stride 0 -> 1; a 1-PE team
    rc, t = split(world, 0, 0, P)
    check(rc == 0 and t and L.shmem_team_n_pes(t) == P and L.shmem_team_my_pe(t) == me, "stride 0")
    if t:
        check(team_sum(t, range(P)), "stride-0 team sum")
        L.shmem_team_destroy(t)
    rc, t = split(world, P - 1, 7, 1)
    check(rc == 0 and (bool(t) == (me == P - 1)), "one-PE team")
    if t:
        check(L.shmem_team_n_pes(t) == 1 and L.shmem_team_translate_pe(t, 0, world) == P - 1,
              "one-PE team shape")
        L.shmem_team_destroy(t)

    # config
    cfg = Config(3)
    rc, t = split(world, 0, 1, P, cfg, NUM_CONTEXTS)
    out = Config(-1)
    check(rc == 0 and L.shmem_team_get_config(t, NUM_CONTEXTS, ctypes.byref(out)) == 0 and
          out.num_contexts == 3, "get_config")
    check(L.shmem_team_get_config(t, 2, ctypes.byref(out)) == -1, "get_config bad mask")
    rc2, t2 = split(world, 0, 1, P, cfg, 2)
    check(rc2 == -1 and not t2, "split bad config mask")
    L.shmem_team_destroy(t)

    # slot pool: 10 slots by default, 3 predefined -> 7 user teams at once
    teams_max = int(os.environ.get("SHMEM_TEAMS_MAX", "10"))
    live = []
    for k in range(teams_max - 3):
        rc, t = split(world, 0, 1, P)
        check(rc == 0 and t, ("pool split", k, rc))
        live.append(t)
    rc, t = split(world, 0, 1, P)
    check(rc == 1 and not t, ("pool exhausted", rc))
    L.shmem_team_destroy(live.pop())
    rc, t = split(world, 0, 1, P)
    check(rc == 0 and t, ("slot reused", rc))
    live.append(t)
    for t in live:
        L.shmem_team_destroy(t)

    # split_2d over the world for every xrange
    for xrange in range(1, P + 2):
        xt, yt = ctypes.c_void_p(0), ctypes.c_void_p(0)
        rc = L.shmem_team_split_2d(world, xrange, None, 0, ctypes.byref(xt), None, 0, ctypes.byref(yt))
        xr = min(xrange, P)
        xstart = me // xr * xr
        xmem = list(range(xstart, min(xstart + xr, P)))
        ymem = list(range(me % xr, P, xr))
        check(rc == 0 and xt.value and yt.value, ("2d", xrange, rc))
        if xt.value and yt.value:
            check(L.shmem_team_n_pes(xt.value) == len(xmem) and
                  L.shmem_team_my_pe(xt.value) == xmem.index(me), ("2d x shape", xrange))
            check(L.shmem_team_n_pes(yt.value) == len(ymem) and
                  L.shmem_team_my_pe(yt.value) == ymem.index(me), ("2d y shape", xrange))
            check(all(L.shmem_team_translate_pe(xt.value, i, world) == pe for i, pe in enumerate(xmem)),
                  ("2d x translate", xrange))
            check(all(L.shmem_team_translate_pe(yt.value, i, world) == pe for i, pe in enumerate(ymem)),
                  ("2d y translate", xrange))
            check(team_sum(xt.value, xmem), ("2d x sum", xrange))
            check(team_sum(yt.value, ymem), ("2d y sum", xrange))
            # a split of a split: every other PE of the y team
            rc, t = split(yt.value, 0, 2, (len(ymem) + 1) // 2)
            sub = ymem[0::2]
            check(rc == 0 and (bool(t) == (me in sub)), ("sub split", xrange))
            if t:
                check(team_sum(t, sub), ("sub sum", xrange))
                L.shmem_team_destroy(t)
            L.shmem_team_destroy(xt.value)
            L.shmem_team_destroy(yt.value)
    S.shmem_barrier_all()
    S.shmem_finalize()
    if bad:
        print(f"PE {me}/{P}: {len(bad)} of {checks} checks FAILED: {bad[:6]}", flush=True)
        return 1
    print(f"PE {me}/{P}: {checks} checks OK", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
