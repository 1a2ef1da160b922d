"""Emit the constexpr model header the HIP kernels are specialised on.

MJX specialises its XLA program on the model structure at ``jit`` time (tree topology,
joint types, collision pairs); the MI355X path does the same at build time: the model
compiler (``mjcf.py``) output is written as a C++ struct of ``static constexpr`` tables,
the kernels are templates over that struct, and every loop over bodies/dofs is fully
unrolled with compile-time indices (registers and immediate LDS offsets instead of
indirect loads). Per-env domain-randomised fields are read from the DR buffer instead
of these constants (``csrc/duck_kernels.hip``).

Usage: ``python -m open_duck_playground_amd.codegen`` (reads the committed assets).
"""

from __future__ import annotations

import os
from typing import List

import numpy as np

from .cabi import model_fingerprint
from .mjcf import JNT_FREE, Model, quat2mat

HERE = os.path.dirname(os.path.abspath(__file__))
# hull/hull SAT tie tolerance (m): axes within it of the best count as ties
HULL_SAT_TIE = 1e-5


def _f(x) -> str:
    x = float(x)
    if x == 0.0:
        return "0.0f"
    r = repr(float(np.float32(x)))
    if "e" not in r and "." not in r and "inf" not in r:
        r += ".0"
    return r + "f"


def _arr(name: str, a, ctype: str) -> str:
    a = np.asarray(a)
    dims = "".join(f"[{d}]" for d in a.shape)
    if a.size == 0:
        dims = "[1]"
        body = "{0}"
        return f"  static constexpr {ctype} {name}{dims} = {body};\n"
    fmt = _f if ctype == "float" else (lambda v: str(int(v)))

    def rec(x):
        if np.ndim(x) == 0:
            return fmt(x)
        return "{" + ", ".join(rec(y) for y in x) + "}"

    return f"  static constexpr {ctype} {name}{dims} = {rec(a)};\n"


def sparse_pattern(m: Model):
    """Row i of M holds its ancestor dofs (incl. itself) in increasing order."""
    rows: List[List[int]] = []
    for i in range(m.nv):
        anc = []
        j = i
        while j >= 0:
            anc.append(j)
            j = m.dof_parentid[j]
        rows.append(sorted(anc))
    adr = np.zeros((m.nv, m.nv), dtype=np.int64) - 1
    k = 0
    for i, r in enumerate(rows):
        for j in r:
            adr[i, j] = k
            k += 1
    return rows, adr, k


def _ancestors(m: Model, k: int, include_self: bool):
    out = [k] if include_self else []
    j = m.dof_parentid[k]
    while j >= 0:
        out.append(j)
        j = m.dof_parentid[j]
    return out


def sparse_code(m: Model, adr) -> str:
    """Straight-line sparse LDL'/solve/matvec on the tree pattern of M (MuJoCo's
    mj_factorM / mj_solveLD / mj_mulM). ``L`` is an accessor (per-thread LDS slice)."""
    nv = m.nv
    o = ["  // M = L' D L, in place: diag holds D, off-diagonals hold L (mj_factorM order)\n",
         "  template <class A> static __device__ __forceinline__ void ldl_factor(const A& L) {\n"]
    for k in range(nv - 1, -1, -1):
        for i in _ancestors(m, k, False):
            o.append(f"    {{ const float t = L[{adr[k, i]}] / L[{adr[k, k]}];")
            for j in _ancestors(m, i, True):
                o.append(f" L[{adr[i, j]}] -= t * L[{adr[k, j]}];")
            o.append(f" L[{adr[k, i]}] = t; }}\n")
        # bound live ranges: the compiler may not carry LDS values in registers across rows
        o.append("    asm volatile(\"\" ::: \"memory\");\n")
    o.append("  }\n")
    o.append("  template <class A> static __device__ __forceinline__ void ldl_solve(const A& L, float* x) {\n")
    for k in range(nv - 1, -1, -1):
        for i in _ancestors(m, k, False):
            o.append(f"    x[{i}] -= L[{adr[k, i]}] * x[{k}];\n")
    for k in range(nv):
        o.append(f"    x[{k}] = x[{k}] / L[{adr[k, k]}];\n")
    for k in range(nv):
        for i in _ancestors(m, k, False):
            o.append(f"    x[{k}] -= L[{adr[k, i]}] * x[{i}];\n")
    o.append("  }\n")
    o.append("  template <class A> static __device__ __forceinline__ void mul_sym(const A& M, const float* x, float* y) {\n")
    for i in range(nv):
        o.append(f"    y[{i}] = 0.0f;\n")
    for i in range(nv):
        for j in sorted(_ancestors(m, i, True)):
            if j == i:
                o.append(f"    y[{i}] += M[{adr[i, i]}] * x[{i}];\n")
            else:
                o.append(f"    {{ const float v = M[{adr[i, j]}]; y[{i}] += v * x[{j}]; y[{j}] += v * x[{i}]; }}\n")
    o.append("  }\n")
    return "".join(o)


def chain_of(m: Model, b: int):
    """dof ancestors of body b (its weld body's dofs and above), increasing"""
    wb = m.body_weldid[b]
    c = []
    if wb > 0:
        j = m.body_dofadr[wb] + m.body_dofnum[wb] - 1
        while j >= 0:
            c.append(int(j))
            j = m.dof_parentid[j]
    return sorted(c)


def _is_anc(m: Model, a: int, b: int) -> bool:
    """body a is b or an ancestor of b"""
    while b > 0:
        if b == a:
            return True
        b = m.body_parentid[b]
    return a == b


def maxchain_of(m: Model):
    return max(len(chain_of(m, b)) for b in range(m.nbody))


def pivot_order(m: Model):
    """Leaves-first elimination order of the dof tree for the register LDL': dofs sorted by
    height (longest path down to a leaf of their subtree), so the limbs' pivots interleave
    (independent dependency chains side by side) while every dof still follows all of its
    descendants. The forward substitution runs it in reverse."""
    nv = m.nv
    h = [0] * nv
    for i in range(nv - 1, -1, -1):
        p = m.dof_parentid[i]
        if p >= 0:
            h[p] = max(h[p], h[i] + 1)
    return sorted(range(nv), key=lambda i: (h[i], -i))


def team_tables(m: Model, rows, adr, pre: str, floor: int):
    """Index tables for the team (16 lanes per env) kernel: lanes pick their work items
    (mass-matrix entries, limb bodies and dofs, constraint rows) from these; they are packed into
    one blob that each launch copies into LDS."""
    nb, nv = m.nbody, m.nv
    full = np.full((nv, nv), -1)
    for i in range(nv):
        for j in rows[i]:
            full[i, j] = full[j, i] = adr[i, j]
    assert nv <= 32
    nc = (nv + 15) // 16
    pplane = [p for p in range(m.npair) if m.pair_geom1[p] == floor]
    pfoot = [p for p in range(m.npair) if m.pair_geom1[p] != floor]
    assert len(pplane) == 2 and len(pfoot) <= 1
    # tree as a root path (bodies up to the first branching body) plus unbranched limbs
    kids = lambda b: [c for c in range(1, nb) if m.body_parentid[c] == b and m.body_weldid[c] != 0]
    root = [1]
    while len(kids(root[-1])) == 1:
        root.append(kids(root[-1])[0])
    branches = []
    for c in kids(root[-1]):
        br = [c]
        while kids(br[-1]):
            assert len(kids(br[-1])) == 1, "limbs must be unbranched"
            br.append(kids(br[-1])[0])
        branches.append(br)
    assert len(branches) <= 16
    brlen = max(len(b) for b in branches)
    br_arr = np.full((len(branches), brlen), -1)
    for i, b in enumerate(branches):
        br_arr[i, :len(b)] = b
    # dofs of each limb body (<= 2: a hinge and its backlash hinge), -1 where absent
    brdof = np.full((len(branches), brlen * 2), -1)
    for i, b in enumerate(branches):
        for d, body in enumerate(b):
            assert m.body_dofnum[body] <= 2
            for jj in range(m.body_dofnum[body]):
                brdof[i, 2 * d + jj] = m.body_dofadr[body] + jj
    # ---- model blob: lane-indexed tables and per-row constraint records, copied into LDS
    # once per launch (int32 words; floats bit-cast) ----
    dt = float(m.opt_timestep)

    def kbi64(solref, solimp, pos):
        tc = max(float(solref[0]), 2.0 * dt)
        dr = float(solref[1])
        dmin = min(max(float(solimp[0]), 1e-4), 0.9999)
        dmax = min(max(float(solimp[1]), 1e-4), 0.9999)
        width = max(1e-15, float(solimp[2]))
        mid = min(max(float(solimp[3]), 1e-4), 0.9999)
        power = max(1.0, float(solimp[4]))
        k = 1.0 / (dmax * dmax * tc * tc * dr * dr)
        b = 2.0 / (dmax * tc)
        x = abs(pos) / width
        if x < mid:
            y = (1.0 / mid ** (power - 1)) * x ** power
        else:
            y = 1 - (1.0 / (1 - mid) ** (power - 1)) * (1 - x) ** power
        imp = min(max(dmin + y * (dmax - dmin), dmin), dmax)
        imp = dmax if x > 1.0 else imp
        return k, b, imp

    f2i = lambda x: int(np.float32(x).view(np.int32))
    blob, boff = [], {}

    def put(name, words):
        boff[name] = len(blob)
        blob.extend(int(w) for w in words)

    put("madr", full.reshape(-1))
    # load_cols: per (column set s, row r, lane) the M entry of column 16 s + lane, or the zero word
    # after M (Lay::MZERO = M + NM) where the tree pattern has none: one unmasked load per entry
    nm_ = int(adr.max()) + 1
    mcolz = np.full((nc, nv, 16), nm_)
    for s_ in range(nc):
        for r in range(nv):
            for ln in range(16):
                c = 16 * s_ + ln
                if c < nv and full[r, c] >= 0:
                    mcolz[s_, r, ln] = full[r, c]
    put("mcolz", mcolz.reshape(-1))
    fric = [i for i in range(nv) if m.dof_frictionloss[i] > 0]
    rec = []
    for i in fric:
        k_, b_, imp = kbi64(m.dof_solref[i], m.dof_solimp[i], 0.0)
        R = max(float(m.dof_invweight0[i]) * (1 - imp) / imp, 1e-15)
        rec += [i, f2i(1.0 / R), f2i(b_)]
    put("fric", rec)  # stride 3: dof, D, b
    # d[0] when the list is d[0], d[0] + 1, ... (an affine map from its index), else -1
    affine = lambda d: d[0] if d and d == list(range(d[0], d[0] + len(d))) else -1
    lim = [j for j in range(m.njnt) if m.jnt_limited[j]]
    rec = []
    for j in lim:
        k_, b_, _ = kbi64(m.jnt_solref[j], m.jnt_solimp[j], 0.0)
        si = m.jnt_solimp[j]
        rec += [m.jnt_dofadr[j], m.jnt_qposadr[j], f2i(m.jnt_range[j][0]), f2i(m.jnt_range[j][1]),
                f2i(m.jnt_margin[j]), f2i(k_), f2i(b_), f2i(m.dof_invweight0[m.jnt_dofadr[j]])] + [f2i(x) for x in si]
    put("lim", rec)  # stride 13: dof, qadr, lo, hi, margin, k, b, invweight, solimp[5]
    slot_of = lambda g: 0 if g == floor else (1 if g == m.id("geom", "left_foot_bottom_tpu") else 2)
    cbody = [m.geom_bodyid[g] for g in (floor, m.id("geom", "left_foot_bottom_tpu"), m.id("geom", "right_foot_bottom_tpu"))]
    rec = []
    for p in range(m.npair):
        s1, s2 = slot_of(m.pair_geom1[p]), slot_of(m.pair_geom2[p])
        tran = float(m.body_invweight0[cbody[s1]][0] + m.body_invweight0[cbody[s2]][0])
        mu = float(m.pair_friction[p][0])
        iw = (tran + mu * mu * tran) * 2.0 * mu * mu / float(m.opt_impratio)
        k_, b_, _ = kbi64(m.pair_solref[p], m.pair_solimp[p], 0.0)
        rec += [s1, s2, f2i(mu), f2i(iw), f2i(m.pair_margin[p]), f2i(k_), f2i(b_), 0] + \
            [f2i(x) for x in m.pair_solimp[p]]
    put("pair", rec)  # stride 13: s1, s2, mu, iw, margin, k, b, pad, solimp[5]
    for name, g in (("chainl", "left_foot_bottom_tpu"), ("chainr", "right_foot_bottom_tpu")):
        c = chain_of(m, m.geom_bodyid[m.id("geom", g)])
        put(name, c + [-1] * (maxchain_of(m) - len(c)))
    put("hull", [f2i(x) for x in np.asarray(m.hulls[0].vert, dtype=np.float64).reshape(-1)])
    # height-field prism SAT (TPhys::collide_hfield / hf_exec): per hull face its outward normal
    # and offset, per hull edge the Gauss-map arc of the negated hull (C = -n_A, D = -n_B), D x C,
    # the edge vector and its first vertex, per hull vertex its position (mesh frame), each vector
    # in its own 16-B record so that one ds_read_b128 fetches it (height-field scenes only; the
    # three tables are contiguous and 16-B aligned: TLay::HT_LDS copies them to LDS when the whole
    # blob does not fit)
    hull = m.hulls[0]
    if int(m.geom_type[floor]) == 1:
        blob.extend([0] * (-len(blob) % 4))
        put("hface", [f2i(x) for f in range(len(hull.face_normal))
                      for x in list(hull.face_normal[f]) + [hull.face_offset[f]]])  # stride 4
        hef = hull_edge_faces(hull)
        rec = []
        for e, (a, b) in enumerate(hull.edge):
            C_, D_ = -np.asarray(hull.face_normal[hef[e][0]]), -np.asarray(hull.face_normal[hef[e][1]])
            v0, v1 = np.asarray(hull.vert[a]), np.asarray(hull.vert[b])
            for v, w in ((C_, 0.0), (D_, 0.0), (np.cross(D_, C_), 0.0), (v1 - v0, float(np.sum((v1 - v0) ** 2))), (v0, 0.0)):
                rec += [f2i(x) for x in v] + [f2i(w)]
        put("hedge", rec)  # stride 20: C, D, D x C, edge (+ |edge|^2), v0 (each padded to 16 B)
        put("hvert", [f2i(x) for v in np.asarray(hull.vert) for x in list(v) + [0.0]])  # stride 4
        boff["hend"] = len(blob)
    else:
        boff["hface"] = boff["hedge"] = boff["hvert"] = boff["hend"] = -1
    d2f, d2l = [-1] * nv, [-1] * nv
    for r, i in enumerate(fric):
        d2f[i] = r
    for r, j in enumerate(lim):
        d2l[m.jnt_dofadr[j]] = r
    put("dof2fric", d2f)
    put("dof2lim", d2l)
    # when the friction / limit rows cover consecutive dofs (the Open Duck scenes: the 14 hinges), the
    # row <-> dof maps are affine and the kernels compute them instead of loading index words (widths,
    # not offsets: B_FRIC0 / B_LIM0 = the first dof, or -1 for the table form)
    lim_dofs = [int(m.jnt_dofadr[j]) for j in lim]
    boff["fric0"] = affine([int(i) for i in fric])
    boff["lim0"] = affine(lim_dofs)
    # flattened tree recursions: per body its dof chain and its subtree, per body the local
    # kinematics record, per dof its body / parent body / first dof of its body / free flag
    mc = maxchain_of(m)
    bchain = np.full((nb, mc), -1)
    for b in range(nb):
        c = chain_of(m, b)
        bchain[b, :len(c)] = c
    dyn = [b for b in range(1, nb) if m.body_weldid[b] != 0]
    sub = [[d for d in dyn if _is_anc(m, b, d)] for b in range(nb)]
    msub = max(len(x) for x in sub)
    bsub = np.full((nb, msub), -1)
    for b in range(nb):
        bsub[b, :len(sub[b])] = sub[b]
    rec = []
    for b in range(nb):
        q, pz = m.body_quat[b], m.body_pos[b]
        nj = int(m.body_jntnum[b]) if b != 1 else 0
        assert nj <= 2
        jr = []
        for jj in range(2):
            if jj < nj:
                j = m.body_jntadr[b] + jj
                jr += [int(m.jnt_qposadr[j])] + [f2i(x) for x in m.jnt_axis[j]]
            else:
                jr += [0, 0, 0, 0]
        rec += [f2i(x) for x in q] + [f2i(x) for x in pz] + [nj] + jr + [0]
    # odd record strides: lane-indexed reads (record per lane) spread over the LDS banks
    put("bkin", rec)  # stride 17: quat4 pos3 njnt (qadr, axis3) x 2, pad
    rec = []
    for i in range(nv):
        b = int(m.dof_bodyid[i])
        rec += [b, int(m.body_parentid[b]), int(m.body_dofadr[b]), int(m.jnt_type[m.dof_jntid[i]] == 0)]
    put("dofrec", rec)  # stride 4: body, parent body, first dof of the body, free-joint flag
    # per-body / joint / actuator / collision-geom / sensor records and the limb tables: every
    # lane-indexed model constant of the substep is read from LDS (no vector-memory loads)
    rec = []
    for b in range(nb):
        rec += [f2i(x) for x in m.body_ipos[b]] + [f2i(x) for x in quat2mat(m.body_iquat[b]).reshape(-1)] + \
            [f2i(x) for x in m.body_inertia[b]] + [int(m.body_weldid[b] != 0), 0]
    put("binert", rec)  # stride 17: ipos3, imat9, inertia3, moving flag, pad
    rec = []
    for j in range(m.njnt):
        rec += [int(m.jnt_bodyid[j]), int(m.jnt_dofadr[j]), int(m.jnt_qposadr[j]), int(m.jnt_type[j])] + \
            [f2i(x) for x in m.jnt_axis[j]] + [0, 0]
    put("jrec", rec)  # stride 9: body, dofadr, qposadr, type, axis3, pad2
    put("damp", [f2i(x) for x in m.dof_damping])
    rec = []
    for a in range(m.nu):
        j = int(m.actuator_trnid[a])
        rec += [int(m.actuator_ctrllimited[a]), f2i(m.actuator_ctrlrange[a][0]), f2i(m.actuator_ctrlrange[a][1]),
                f2i(m.actuator_gear[a]), int(m.jnt_qposadr[j]), int(m.jnt_dofadr[j]), f2i(m.actuator_kv[a]),
                int(m.actuator_forcelimited[a]), f2i(m.actuator_forcerange[a][0]), f2i(m.actuator_forcerange[a][1]),
                0, 0]
    put("act", rec)  # stride 12: ctrllimited, ctrlrange2, gear, qadr, dof, kv, forcelimited, forcerange2, pad2
    # affine index maps (see B_FRIC0): actuator -> dof / qpos address, limit row -> qpos address, and
    # dof -> body (the first B_DBN dofs on body B_DB0, then body = dof + B_DBD; B_DBD = -1000: table)
    act_j = [int(m.actuator_trnid[a]) for a in range(m.nu)]
    boff["actd0"] = affine([int(m.jnt_dofadr[j]) for j in act_j])
    boff["actq0"] = affine([int(m.jnt_qposadr[j]) for j in act_j])
    boff["limq0"] = affine([int(m.jnt_qposadr[j]) for j in lim])
    db = [int(x) for x in m.dof_bodyid]
    nfr = 6 if (m.njnt > 0 and m.jnt_type[0] == 0 and m.jnt_dofadr[0] == 0) else 0
    ok = nv > nfr and all(db[i] == db[0] for i in range(nfr)) and \
        all(db[i] == i + (db[nfr] - nfr) for i in range(nfr, nv))
    boff["dbn"] = nfr
    boff["db0"] = db[0] if nfr else 0
    boff["dbd"] = (db[nfr] - nfr) if ok else -1000
    # joints after a leading free joint: all hinges with body / dof / qpos address = j + const
    # (B_JAFF = 1; com_pos and Euler then compute them instead of loading the joint records)
    j0 = 1 if (m.njnt > 0 and m.jnt_type[0] == 0) else 0
    js = range(j0, m.njnt)
    jb, jd, jq = ([int(a[j]) - j for j in js] for a in (m.jnt_bodyid, m.jnt_dofadr, m.jnt_qposadr))
    jaff = len(js) > 0 and all(int(m.jnt_type[j]) == 3 for j in js) and len(set(jb)) == 1 and \
        len(set(jd)) == 1 and len(set(jq)) == 1
    boff["jaff"] = 1 if jaff else 0
    boff["jn0"] = j0
    boff["jbd"], boff["jdd"], boff["jqd"] = (jb[0], jd[0], jq[0]) if jaff else (0, 0, 0)
    rec = []
    for g in (floor, m.id("geom", "left_foot_bottom_tpu"), m.id("geom", "right_foot_bottom_tpu")):
        rec += [int(m.geom_bodyid[g])] + [f2i(x) for x in m.geom_pos[g]] + \
            [f2i(x) for x in quat2mat(m.geom_quat[g]).reshape(-1)] + [0, 0, 0]
    put("cgeom", rec)  # stride 16: body, pos3, mat9, pad3 (slots: floor, left foot, right foot)
    rec = []
    for i in range(m.nsensor):
        st = int(m.sensor_objid[i])
        rec += [int(m.sensor_type[i]), st, int(m.sensor_adr[i]), int(m.site_bodyid[st])] + \
            [f2i(x) for x in m.site_pos[st]] + [f2i(x) for x in quat2mat(m.site_quat[st]).reshape(-1)] + \
            [f2i(x) for x in m.site_quat[st]]
    put("sens", rec)  # stride 20: type, site, adr, body, spos3, smat9, squat4
    # nominal per-env model block, in Lay order DMASS (nb), DIPOS (3), DARM, DFRIC (nv), DQ0 (nq), DKP (nu)
    put("nom", [f2i(x) for x in np.concatenate([m.body_mass, m.body_ipos[1], m.dof_armature, m.dof_frictionloss,
                                                 m.qpos0, m.actuator_kp])])
    put("br", br_arr.reshape(-1))  # [T_NBR][T_BRLEN] limb bodies
    put("brdof", brdof.reshape(-1))  # [T_NBR][2 T_BRLEN] their dofs
    dch = np.full((nv, mc), -1)
    for i in range(nv):
        c = sorted(_ancestors(m, i, True))
        dch[i, :len(c)] = c
    put("dchain", dch.reshape(-1))  # ancestors of dof i incl. itself, ascending (= M row order)
    # the same chains as "free-joint dofs, then a run of consecutive limb dofs up to i" (B_DCHAFF = 1):
    # crb computes them from the run starts T_DLST instead of loading index words
    nfd = 6 if (m.njnt > 0 and m.jnt_type[0] == 0 and m.jnt_dofadr[0] == 0) else 0
    dlst = [i for i in range(nfd, nv) if i == nfd or (mc > nfd and dch[i, nfd] == i)]

    def chain_model(i):
        if i < nfd:
            return list(range(i + 1))
        st = max(x for x in dlst if x <= i)
        return list(range(nfd)) + list(range(st, i + 1))
    dchaff = nfd > 0 and len(dlst) > 0 and all(
        [int(x) for x in dch[i] if x >= 0] == chain_model(i) for i in range(nv))
    boff["dchaff"] = 1 if dchaff else 0
    boff["dchn"] = nfd
    put("mrow", [adr[i, min(_ancestors(m, i, True))] for i in range(nv)])  # adr of row i's first entry
    extra_const = [f"  static constexpr int T_MAXSUB = {msub};\n"]
    T = lambda name, a, t: f"__device__ const {t} {pre}_{name}{''.join(f'[{d}]' for d in np.shape(a))} = " + \
        _arr("x", np.asarray(a), t).split("= ", 1)[1]
    # the lane-indexed tables live in the blob (copied to LDS per launch); it is the only device array
    tabs = {"blob": (np.array(blob, dtype=np.int64), "int")}
    dev = [T(k, a, t) for k, (a, t) in tabs.items()]
    acc = [f"  static constexpr int PLANE_PAIR[2] = {{{pplane[0]}, {pplane[1]}}};\n",
           f"  static constexpr int FOOT_PAIR = {pfoot[0] if pfoot else -1};\n",
           _arr("T_PORD", pivot_order(m), "int"),
           f"  static constexpr int T_NROOT = {len(root)}, T_NBR = {len(branches)}, T_BRLEN = {brlen}, "
           f"T_BRMD = {int(max(m.body_dofnum[b] for br in branches for b in br))};\n",
           _arr("T_ROOT", root, "int"),
           _arr("T_BRB", br_arr, "int"),  # [T_NBR][T_BRLEN] limb bodies, -1 past a limb's end
           _arr("T_DLST", dlst if dlst else [0], "int"),  # starts of the consecutive limb-dof runs (B_DCHAFF)
           f"  static constexpr int T_NDLST = {len(dlst)};\n",
           f"  static constexpr int NBLOB = {len(blob)};\n"] + extra_const + [
           "".join(f"  static constexpr int B_{k.upper()} = {v};\n" for k, v in boff.items())]
    for k, (a, t) in tabs.items():
        shp = np.shape(a)
        if len(shp) == 1:
            acc.append(f"  static __device__ __forceinline__ const {t}* t_{k}() {{ return {pre}_{k}; }}\n")
        else:
            acc.append(f"  static __device__ __forceinline__ const {t} (*t_{k}())[{shp[1]}] {{ return {pre}_{k}; }}\n")
    return dev, acc


def silhouette_cap(hull, hef, n_dir: int = 20000) -> int:
    """The most hull edges on one silhouette (edges whose two faces lie on opposite sides of a
    plane through the hull's Gauss map centre), over a Fibonacci sphere of view directions, plus
    a margin of 4: the capacity of TPhys::collide_hfield's per-foot silhouette list."""
    i = np.arange(n_dir) + 0.5
    zz = 1 - 2 * i / n_dir
    ph = np.pi * (1 + 5 ** 0.5) * i
    r = np.sqrt(1 - zz * zz)
    d = np.stack([r * np.cos(ph), r * np.sin(ph), zz], axis=1)
    fn = np.asarray(hull.face_normal, dtype=np.float64)
    sa, sb = d @ fn[hef[:, 0]].T, d @ fn[hef[:, 1]].T
    return int(((sa * sb) < 0).sum(axis=1).max()) + 4


def hull_edge_faces(hull) -> np.ndarray:
    """The two faces adjacent to each hull edge (from the merged polygons): edge e is the
    Gauss-map arc between the normals of faces [e][0] and [e][1] — the edge-pair filter of the
    hull/hull SAT (oracle/duck_oracle.c derives the same table from the face planes)."""
    adj = {}
    for f, poly in enumerate(hull.face_vert):
        for i in range(len(poly)):
            a, b = poly[i], poly[(i + 1) % len(poly)]
            adj.setdefault((min(a, b), max(a, b)), []).append(f)
    out = [sorted(adj[(int(a), int(b))]) for a, b in hull.edge]
    assert all(len(x) == 2 for x in out), "every hull edge must join exactly two faces"
    return np.array(out, dtype=np.int64)


def model_header(m: Model, variant: str) -> str:
    nb, nv, nq, nu, nj = m.nbody, m.nv, m.nq, m.nu, m.njnt
    rows, adr, nm = sparse_pattern(m)
    # chains: for each body, its dof ancestors (ordered increasing)
    chain = []
    for b in range(nb):
        wb = m.body_weldid[b]
        c = []
        if wb > 0:
            j = m.body_dofadr[wb] + m.body_dofnum[wb] - 1
            while j >= 0:
                c.append(j)
                j = m.dof_parentid[j]
        chain.append(sorted(c))
    maxchain = max(len(c) for c in chain)
    chain_arr = np.full((nb, maxchain), -1)
    for b, c in enumerate(chain):
        chain_arr[b, :len(c)] = c
    hull = m.hulls[0]
    floor = m.id("geom", "floor")
    lfoot = m.id("geom", "left_foot_bottom_tpu")
    rfoot = m.id("geom", "right_foot_bottom_tpu")
    body_imat = np.array([quat2mat(q) for q in m.body_iquat])
    site_mat = np.array([quat2mat(q) for q in m.site_quat])
    geom_mat = np.array([quat2mat(q) for q in m.geom_quat])
    free = [j for j in range(nj) if m.jnt_type[j] == JNT_FREE]
    assert free == [0] and m.body_jntadr[1] == 0, "kernel assumes body 1 carries the free joint"
    for j in range(nj):
        if j not in free:
            assert np.allclose(m.jnt_pos[j], 0), "kernel assumes hinge anchors at the body origin"
            assert np.allclose(m.jnt_axis[j], m.jnt_axis[m.body_jntadr[m.jnt_bodyid[j]]]), "same-axis joints per body"
    assert m.nsite <= 8 and len(m.hulls) == 1
    hc = hull.vert.mean(axis=0)
    hr = float(np.max(np.linalg.norm(hull.vert - hc, axis=1)))
    hef = hull_edge_faces(hull)
    # height field: the most grid cells the hull's bounding box can span along x / y in any
    # orientation, floor(diameter / cell) + 2 (the prism loop's static bound)
    diam = float(np.max(np.linalg.norm(hull.vert[:, None, :] - hull.vert[None, :, :], axis=2)))
    if int(m.hfield_nrow) > 1 and int(m.hfield_ncol) > 1:
        cell = (2 * float(m.hfield_size[0]) / (int(m.hfield_ncol) - 1), 2 * float(m.hfield_size[1]) / (int(m.hfield_nrow) - 1))
        hf_cells = tuple(min(int(diam // c) + 2, n - 1) for c, n in zip(cell, (int(m.hfield_ncol), int(m.hfield_nrow))))
    else:
        hf_cells = (1, 1)
    pre = f"DuckModel_{variant}"
    maxfv = max(len(f) for f in hull.face_vert)
    fvert = np.full((len(hull.face_vert), maxfv), -1, dtype=np.int64)
    for j, f in enumerate(hull.face_vert):
        fvert[j, :len(f)] = f
    dev = [f"__device__ const int {pre}_hull_face_vert_d[{len(hull.face_vert)}][{maxfv}] = {_arr('x', fvert, 'int').split('= ', 1)[1]}",
           f"__device__ const int {pre}_hull_face_nv_d[{len(hull.face_vert)}] = {_arr('x', [len(f) for f in hull.face_vert], 'int').split('= ', 1)[1]}",
f"__device__ const float {pre}_hull_vert_d[{len(hull.vert)}][3] = {_arr('x', hull.vert, 'float').split('= ', 1)[1]}",
           f"__device__ const float {pre}_hull_face_normal_d[{len(hull.face_normal)}][3] = {_arr('x', hull.face_normal, 'float').split('= ', 1)[1]}",
           f"__device__ const float {pre}_hull_face_offset_d[{len(hull.face_offset)}] = {_arr('x', hull.face_offset, 'float').split('= ', 1)[1]}",
           f"__device__ const int {pre}_hull_edge_d[{len(hull.edge)}][2] = {_arr('x', hull.edge, 'int').split('= ', 1)[1]}",
           f"__device__ const int {pre}_hull_edge_face_d[{len(hef)}][2] = {_arr('x', hef, 'int').split('= ', 1)[1]}",
           f"__device__ const int {pre}_chain_d[{nb}][{maxchain}] = {_arr('x', chain_arr, 'int').split('= ', 1)[1]}"]
    acc = [f"  static constexpr int HULL_MAXFV = {maxfv};  // most vertices of a hull face polygon\n",
           f"  static __device__ __forceinline__ const int (*hull_face_vert_d())[{maxfv}] {{ return {pre}_hull_face_vert_d; }}\n",
           f"  static __device__ __forceinline__ const int* hull_face_nv_d() {{ return {pre}_hull_face_nv_d; }}\n",
           f"  static __device__ __forceinline__ const float (*hull_vert_d())[3] {{ return {pre}_hull_vert_d; }}\n",
           f"  static __device__ __forceinline__ const float (*hull_face_normal_d())[3] {{ return {pre}_hull_face_normal_d; }}\n",
           f"  static __device__ __forceinline__ const float* hull_face_offset_d() {{ return {pre}_hull_face_offset_d; }}\n",
           f"  static __device__ __forceinline__ const int (*hull_edge_d())[2] {{ return {pre}_hull_edge_d; }}\n",
           f"  static __device__ __forceinline__ const int (*hull_edge_face_d())[2] {{ return {pre}_hull_edge_face_d; }}\n",
           f"  static __device__ __forceinline__ const int (*chain_d())[{maxchain}] {{ return {pre}_chain_d; }}\n"]
    out = [f"// generated by open_duck_playground_amd/codegen.py from assets/{m.name} — do not edit\n",
           "#pragma once\n\n"] + dev + [
           f"struct DuckModel_{variant} {{\n"] + acc + [
           f"  static constexpr int NB = {nb}, NQ = {nq}, NV = {nv}, NU = {nu}, NJ = {nj}, NSITE = {m.nsite};\n",
           f"  static constexpr int NM = {nm}, MAXCHAIN = {maxchain}, NSENSORDATA = {m.nsensordata};\n",
           f"  static constexpr int NHV = {len(hull.vert)}, NHF = {len(hull.face_normal)}, NHE = {len(hull.edge)};\n",
           f"  static constexpr int FLOOR_GEOM = {floor}, LFOOT_GEOM = {lfoot}, RFOOT_GEOM = {rfoot};\n",
           f"  static constexpr int LFOOT_BODY = {m.geom_bodyid[lfoot]}, RFOOT_BODY = {m.geom_bodyid[rfoot]};\n",
           f"  static constexpr int FLOOR_TYPE = {m.geom_type[floor]};\n",
           f"  static constexpr int HF_NROW = {int(m.hfield_nrow)}, HF_NCOL = {int(m.hfield_ncol)};\n",
           f"  static constexpr float HF_SIZE[4] = {{{', '.join(_f(x) for x in m.hfield_size)}}};\n",
           f"  static constexpr int HF_MAXCX = {hf_cells[0]}, HF_MAXCY = {hf_cells[1]};  // cells a hull's box spans\n",
           f"  static constexpr float timestep = {_f(m.opt_timestep)}, impratio = {_f(m.opt_impratio)};\n",
           f"  static constexpr float tolerance = {_f(m.opt_tolerance)}, ls_tolerance = {_f(m.opt_ls_tolerance)};\n",
           f"  static constexpr float meaninertia = {_f(m.stat_meaninertia)};\n",
           f"  static constexpr int iterations = {m.opt_iterations}, ls_iterations = {m.opt_ls_iterations};\n",
           f"  static constexpr float hull_radius = {_f(hr)};\n",
           f"  static constexpr float HULL_SAT_TIE = {_f(HULL_SAT_TIE)};  // = DUCK_HULL_SAT_TIE, oracle/duck_oracle.c\n",
           f"  // duck_model_fingerprint of the model this header bakes: duck_create binds a model to it\n",
           f"  static constexpr unsigned long long FINGERPRINT = 0x{model_fingerprint(m):016x}ull;\n",
           ]
    out.append(_arr("gravity", m.opt_gravity, "float"))
    out.append(_arr("hull_center", hc, "float"))
    # the hull's box in its mesh frame (conservative prefilter of the foot/foot SAT)
    out.append(_arr("hull_box_c", 0.5 * (hull.vert.min(axis=0) + hull.vert.max(axis=0)), "float"))
    out.append(_arr("hull_box_h", 0.5 * (hull.vert.max(axis=0) - hull.vert.min(axis=0)), "float"))
    for name in ("body_parentid", "body_jntnum", "body_jntadr", "body_dofnum", "body_dofadr", "body_weldid"):
        out.append(_arr(name, m.arrays[name], "int"))
    for name in ("body_pos", "body_quat", "body_ipos", "body_mass", "body_inertia", "body_invweight0"):
        out.append(_arr(name, m.arrays[name], "float"))
    out.append(_arr("body_imat", body_imat.reshape(nb, 9), "float"))
    for name in ("jnt_type", "jnt_qposadr", "jnt_dofadr", "jnt_bodyid", "jnt_limited"):
        out.append(_arr(name, m.arrays[name], "int"))
    for name in ("jnt_pos", "jnt_axis", "jnt_range", "jnt_margin", "jnt_solref", "jnt_solimp"):
        out.append(_arr(name, m.arrays[name], "float"))
    for name in ("dof_bodyid", "dof_jntid", "dof_parentid"):
        out.append(_arr(name, m.arrays[name], "int"))
    for name in ("dof_armature", "dof_damping", "dof_frictionloss", "dof_invweight0", "dof_solref", "dof_solimp"):
        out.append(_arr(name, m.arrays[name], "float"))
    out.append(_arr("qpos0", m.qpos0, "float"))
    out.append(_arr("site_bodyid", m.site_bodyid, "int"))
    out.append(_arr("site_pos", m.site_pos, "float"))
    out.append(_arr("site_quat", m.site_quat, "float"))
    out.append(_arr("site_mat", site_mat.reshape(-1, 9), "float"))
    out.append(_arr("cgeom_body", m.geom_bodyid[[floor, lfoot, rfoot]], "int"))
    out.append(_arr("geom_pos", m.geom_pos[[floor, lfoot, rfoot]], "float"))
    out.append(_arr("geom_mat", geom_mat[[floor, lfoot, rfoot]].reshape(3, 9), "float"))
    out.append(_arr("actuator_trnid", m.actuator_trnid, "int"))
    for name in ("actuator_kp", "actuator_kv", "actuator_gear", "actuator_ctrlrange", "actuator_forcerange"):
        out.append(_arr(name, m.arrays[name], "float"))
    out.append(_arr("actuator_ctrllimited", m.actuator_ctrllimited, "int"))
    out.append(_arr("actuator_forcelimited", m.actuator_forcelimited, "int"))
    out.append(_arr("actuator_dof", [m.jnt_dofadr[j] for j in m.actuator_trnid], "int"))
    out.append(_arr("actuator_qadr", [m.jnt_qposadr[j] for j in m.actuator_trnid], "int"))
    out.append(f"  static constexpr int NSENSOR = {m.nsensor}, IMU_SITE = {m.id('site', 'imu')};\n")
    out.append(f"  static constexpr int LFOOT_SITE = {m.id('site', 'left_foot')}, RFOOT_SITE = {m.id('site', 'right_foot')};\n")
    acc_sites = [m.sensor_objid[i] for i in range(m.nsensor) if m.sensor_type[i] == 2]
    assert all(m.site_bodyid[s] == 1 for s in acc_sites), "accelerometer must sit on the free body"
    out.append(_arr("sensor_type", m.sensor_type, "int"))
    out.append(_arr("sensor_objid", m.sensor_objid, "int"))
    out.append(_arr("sensor_adr", m.sensor_adr, "int"))
    # collision pairs in slot order: pair p -> contact slots 4p..4p+3
    out.append(f"  static constexpr int NPAIR = {m.npair};\n")
    out.append(_arr("pair_geom1", m.pair_geom1, "int"))
    out.append(_arr("pair_geom2", m.pair_geom2, "int"))
    out.append(_arr("pair_friction", m.pair_friction, "float"))
    out.append(_arr("pair_solref", m.pair_solref, "float"))
    out.append(_arr("pair_solimp", m.pair_solimp, "float"))
    out.append(_arr("pair_margin", m.pair_margin, "float"))
    out.append(_arr("hull_vert", hull.vert, "float"))
    out.append(_arr("hull_face_normal", hull.face_normal, "float"))
    out.append(_arr("hull_face_offset", hull.face_offset, "float"))
    out.append(_arr("hull_edge", hull.edge, "int"))
    # the height field's per-lane prism SAT (TPhys::hf_exec): per hull edge its two faces (the
    # Gauss-map arc C = -n_a -> D = -n_b) and D x C; HF_SILCAP bounds the edges on a silhouette
    fnrm = np.asarray(hull.face_normal, dtype=np.float64)
    out.append(_arr("hull_edge_face", hef, "int"))
    out.append(_arr("hull_edge_dxc", np.cross(-fnrm[hef[:, 1]], -fnrm[hef[:, 0]]), "float"))
    out.append(f"  static constexpr int HF_SILCAP = {silhouette_cap(hull, hef)};\n")
    # sparse mass-matrix pattern
    out.append(_arr("M_adr", adr, "int"))
    out.append(_arr("M_rowlen", [len(r) for r in rows], "int"))
    out.append(_arr("chain", chain_arr, "int"))
    out.append(_arr("chain_len", [len(c) for c in chain], "int"))
    fric = [i for i in range(nv) if m.dof_frictionloss[i] > 0]
    lim = [j for j in range(nj) if m.jnt_limited[j]]
    out.append(f"  static constexpr int NFRIC = {len(fric)}, NLIM = {len(lim)};\n")
    out.append(_arr("fric_dof", fric, "int"))
    out.append(_arr("lim_jnt", lim, "int"))
    out.append(sparse_code(m, adr))
    tdev, tacc = team_tables(m, rows, adr, pre, floor)
    out.extend(tacc)
    out.append("};\n")
    return "".join(out[:2] + tdev + out[2:])


# the scenes libduck.so ships with: (variant name, task asset)
DEFAULT_VARIANTS = (("flat", "flat_terrain"), ("backlash", "flat_terrain_backlash"), ("rough", "rough_terrain"),
                    ("rough_backlash", "rough_terrain_backlash"))


def variant_unit(variant: str, header: str) -> str:
    """The translation unit of one compiled model: the kernel templates instantiated on its header."""
    return (f"// variant_{variant}.hip — kernels for the '{variant}' model ({header}).\n"
            f"#include \"duck_env_kernels.h\"\n#include \"{header}\"\n\n"
            f"DUCK_DEFINE_VARIANT({variant}, DuckModel_{variant})\n")


def variant_registry(variants) -> str:
    """duck_variants.inc: the X-macro list duck_capi.hip builds its variant table from."""
    return "// generated by open_duck_playground_amd/codegen.py — do not edit\n" + \
        "".join(f"DUCK_VARIANT({v})\n" for v in variants)


def main():
    gen = os.path.join(HERE, "csrc", "generated")
    os.makedirs(gen, exist_ok=True)
    for variant, task in DEFAULT_VARIANTS:
        m = Model.load(os.path.join(HERE, "assets", f"{task}.npz"))
        with open(os.path.join(gen, f"duck_model_{variant}.h"), "w") as f:
            f.write(model_header(m, variant))
    with open(os.path.join(gen, "duck_variants.inc"), "w") as f:
        f.write(variant_registry([v for v, _ in DEFAULT_VARIANTS]))


if __name__ == "__main__":
    main()
