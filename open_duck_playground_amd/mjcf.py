"""MJCF compiler for the Open Duck Mini v2 scenes (host side, runs once per task).

This is the build's replacement for the two upstream calls the reference makes at
env construction:

* ``mujoco.MjModel.from_xml_string(xml, assets=get_assets())``
  (``playground/open_duck_mini_v2/base.py:53-55``), and
* ``mjx.put_model`` (``base.py:61``),

restricted to the MJCF subset the four Open Duck scenes use
(``xmls/scene_flat_terrain.xml``, ``scene_flat_terrain_backlash.xml``,
``scene_rough_terrain_backlash.xml`` and the robot files they include):
``<include>``, nested ``<default>`` classes with ``childclass`` inheritance, bodies with
``pos``/``quat``, ``<inertial fullinertia=...>``, ``<freejoint>``/hinge joints,
mesh/plane/hfield geoms, sites, ``<position>`` actuators with ``inheritrange``,
the 15 site sensors of ``open_duck_mini_v2.xml:26-42`` and keyframes.

It emits a flat dict of numpy arrays (``Model``) that is (a) consumed by the CPU oracle
through the C model descriptor (``include/duck_model.h``) and (b) turned into the
constexpr model header the HIP kernels are specialised on (``codegen.py``).

Semantics follow MuJoCo's compiler (documented behaviour, re-derived here):

* hinge joints are ``limited`` when a range is given (``autolimits`` default),
* actuators with ``inheritrange="1"`` get ``ctrlrange`` = the joint range, and
  ``ctrllimited``/``forcelimited`` are on when the corresponding range is set,
* ``fullinertia`` is diagonalised into ``body_inertia`` + ``body_iquat``,
* collision meshes are replaced by their convex hull (qhull, as MuJoCo does),
* contact pairs come from ``contype``/``conaffinity`` with parent-child filtering and
  contact parameters are mixed by ``priority`` (higher priority wins) else max/mean,
* ``dof_invweight0``/``body_invweight0``/``stat.meaninertia`` are computed at ``qpos0``
  like ``mj_setConst`` (``set0``).
"""

from __future__ import annotations

import os
import struct
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

# enum values follow mjtJoint / mjtGeom / mjtSensor naming (values are ours)
JNT_FREE, JNT_BALL, JNT_SLIDE, JNT_HINGE = 0, 1, 2, 3
GEOM_PLANE, GEOM_HFIELD, GEOM_SPHERE, GEOM_CAPSULE, GEOM_ELLIPSOID, GEOM_CYLINDER, GEOM_BOX, GEOM_MESH = range(8)
GEOM_TYPES = {"plane": GEOM_PLANE, "hfield": GEOM_HFIELD, "sphere": GEOM_SPHERE, "capsule": GEOM_CAPSULE,
              "ellipsoid": GEOM_ELLIPSOID, "cylinder": GEOM_CYLINDER, "box": GEOM_BOX, "mesh": GEOM_MESH}

SENS_GYRO, SENS_VELOCIMETER, SENS_ACCELEROMETER, SENS_FRAMEZAXIS, SENS_FRAMEXAXIS, SENS_FRAMELINVEL, \
    SENS_FRAMEANGVEL, SENS_FRAMEPOS, SENS_FRAMEQUAT = range(9)
SENSOR_TYPES = {"gyro": (SENS_GYRO, 3), "velocimeter": (SENS_VELOCIMETER, 3),
                "accelerometer": (SENS_ACCELEROMETER, 3), "framezaxis": (SENS_FRAMEZAXIS, 3),
                "framexaxis": (SENS_FRAMEXAXIS, 3), "framelinvel": (SENS_FRAMELINVEL, 3),
                "frameangvel": (SENS_FRAMEANGVEL, 3), "framepos": (SENS_FRAMEPOS, 3),
                "framequat": (SENS_FRAMEQUAT, 4)}

MJMINVAL = 1e-15

_DEFAULT_JOINT = {"type": "hinge", "pos": "0 0 0", "axis": "0 0 1", "damping": "0", "frictionloss": "0",
                  "armature": "0", "limited": "auto", "range": None, "margin": "0",
                  "solreflimit": "0.02 1", "solimplimit": "0.9 0.95 0.001 0.5 2",
                  "solreffriction": "0.02 1", "solimpfriction": "0.9 0.95 0.001 0.5 2"}
_DEFAULT_GEOM = {"type": "sphere", "pos": "0 0 0", "quat": "1 0 0 0", "contype": "1", "conaffinity": "1",
                 "condim": "3", "priority": "0", "friction": "1 0.005 0.0001", "solref": "0.02 1",
                 "solimp": "0.9 0.95 0.001 0.5 2", "margin": "0", "gap": "0", "size": "0 0 0", "group": "0",
                 "solmix": "1"}
_DEFAULT_POSITION = {"kp": "1", "kv": "0", "ctrlrange": None, "forcerange": None, "ctrllimited": "auto",
                     "forcelimited": "auto", "inheritrange": "0", "gear": "1"}
_DEFAULT_SITE = {"pos": "0 0 0", "quat": "1 0 0 0"}


def _vec(s, n=None, dtype=float):
    if s is None:
        return None
    v = np.array([dtype(x) for x in s.split()], dtype=np.float64 if dtype is float else np.int64)
    if n is not None and v.size != n:
        raise ValueError(f"expected {n} values, got {s!r}")
    return v


# --------------------------------------------------------------------------------------
# quaternion / rotation helpers (w, x, y, z convention, as MuJoCo)
# --------------------------------------------------------------------------------------

def quat_normalize(q):
    q = np.asarray(q, dtype=np.float64)
    n = np.linalg.norm(q)
    return q / n if n > MJMINVAL else np.array([1.0, 0, 0, 0])


def quat_mul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
                     w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                     w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


def quat2mat(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def mat2quat(R):
    # Shepperd's method, returns w >= 0
    t = np.trace(R)
    if t > 0:
        s = np.sqrt(t + 1.0) * 2
        q = np.array([0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s])
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        q = np.array([(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s])
    elif R[1, 1] > R[2, 2]:
        s = np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        q = np.array([(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s])
    else:
        s = np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        q = np.array([(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s])
    if q[0] < 0:
        q = -q
    return quat_normalize(q)


def axis_angle_quat(axis, angle):
    axis = np.asarray(axis, dtype=np.float64)
    s = np.sin(angle / 2)
    return np.array([np.cos(angle / 2), axis[0] * s, axis[1] * s, axis[2] * s])


# --------------------------------------------------------------------------------------
# asset readers
# --------------------------------------------------------------------------------------

def read_stl(path: str) -> np.ndarray:
    """Binary (or ASCII) STL -> unique vertex array (MuJoCo merges duplicate vertices)."""
    with open(path, "rb") as f:
        data = f.read()
    verts = None
    if len(data) >= 84:
        ntri = struct.unpack("<I", data[80:84])[0]
        if 84 + 50 * ntri == len(data):
            rec = np.frombuffer(data[84:], dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]))
            verts = rec["v"].reshape(-1, 3).astype(np.float64)
    if verts is None:
        pts = []
        for line in data.decode("ascii", "replace").splitlines():
            line = line.strip()
            if line.startswith("vertex"):
                pts.append([float(x) for x in line.split()[1:4]])
        verts = np.array(pts, dtype=np.float64)
    # MuJoCo stores mesh vertices as float32
    verts = verts.astype(np.float32).astype(np.float64)
    _, idx = np.unique(verts, axis=0, return_index=True)
    return verts[np.sort(idx)]


@dataclass
class Hull:
    vert: np.ndarray          # (nv, 3) hull vertices (geom frame)
    face_normal: np.ndarray   # (nf, 3) outward unit normals of hull faces
    face_offset: np.ndarray   # (nf,)   n . x = offset on the face plane
    face_vert: List[List[int]]  # polygon vertex indices (CCW seen from outside)
    edge: np.ndarray          # (ne, 2) unique hull edges (vertex index pairs)


def convex_hull(points: np.ndarray) -> Hull:
    """Convex hull with coplanar triangles merged into polygons (qhull, as MuJoCo)."""
    from scipy.spatial import ConvexHull
    h = ConvexHull(points)
    keep = np.array(sorted(set(h.vertices.tolist())))
    remap = -np.ones(len(points), dtype=np.int64)
    remap[keep] = np.arange(len(keep))
    vert = points[keep]
    # group simplices by plane
    groups: List[Tuple[np.ndarray, float, List[np.ndarray]]] = []
    for simplex, eq in zip(h.simplices, h.equations):
        n, off = eq[:3], -eq[3]
        for g in groups:
            if np.dot(g[0], n) > 1 - 1e-9 and abs(g[1] - off) < 1e-9:
                g[2].append(simplex)
                break
        else:
            groups.append((n, off, [simplex]))
    face_normal, face_offset, face_vert = [], [], []
    edges = set()
    for n, off, simplices in groups:
        # boundary edges of the merged polygon (edges used by exactly one triangle of the group)
        cnt: Dict[Tuple[int, int], int] = {}
        for s in simplices:
            s = [int(remap[i]) for i in s]
            for a, b in ((s[0], s[1]), (s[1], s[2]), (s[2], s[0])):
                k = (min(a, b), max(a, b))
                cnt[k] = cnt.get(k, 0) + 1
        bnd = [k for k, c in cnt.items() if c == 1]
        edges.update(bnd)
        vids = sorted(set(v for k in bnd for v in k))
        # order polygon CCW around the outward normal
        c = vert[vids].mean(axis=0)
        u = vert[vids[0]] - c
        u /= np.linalg.norm(u)
        w = np.cross(n, u)
        ang = [np.arctan2(np.dot(vert[v] - c, w), np.dot(vert[v] - c, u)) for v in vids]
        vids = [v for _, v in sorted(zip(ang, vids))]
        face_normal.append(n / np.linalg.norm(n))
        face_offset.append(off)
        face_vert.append(vids)
    return Hull(vert=vert, face_normal=np.array(face_normal), face_offset=np.array(face_offset),
                face_vert=face_vert, edge=np.array(sorted(edges), dtype=np.int64))


def read_hfield_png(path: str) -> np.ndarray:
    """Height field image -> (nrow, ncol) elevation in [0, 1].

    Grey value (the three channels are equal in ``hfield.png``), rows flipped so row 0
    is at -y, normalised by (v - min) / (max - min) as MuJoCo's hfield compiler does.
    """
    from PIL import Image
    img = np.asarray(Image.open(path).convert("L"), dtype=np.float64)
    img = img[::-1, :]
    lo, hi = img.min(), img.max()
    return (img - lo) / (hi - lo) if hi > lo else np.zeros_like(img)


# --------------------------------------------------------------------------------------
# XML loading with includes and defaults
# --------------------------------------------------------------------------------------

def _load_tree(path: str) -> ET.Element:
    root = ET.parse(path).getroot()
    base = os.path.dirname(path)

    def expand(el: ET.Element):
        out = []
        for child in list(el):
            if child.tag == "include":
                inc = _load_tree(os.path.join(base, child.get("file")))
                out.extend(list(inc))
            else:
                expand(child)
                out.append(child)
        for c in list(el):
            el.remove(c)
        for c in out:
            el.append(c)

    expand(root)
    # merge duplicate top-level sections (MuJoCo allows several <worldbody>, <default>, ...)
    return root


class _Defaults:
    def __init__(self):
        self.classes: Dict[str, Dict[str, Dict[str, str]]] = {
            "main": {"joint": dict(_DEFAULT_JOINT), "geom": dict(_DEFAULT_GEOM),
                     "position": dict(_DEFAULT_POSITION), "site": dict(_DEFAULT_SITE)}}

    def parse(self, el: ET.Element, parent: str = "main"):
        name = el.get("class", "main")
        if name not in self.classes:
            self.classes[name] = {k: dict(v) for k, v in self.classes[parent].items()}
        for child in el:
            if child.tag == "default":
                self.parse(child, name)
            else:
                self.classes[name].setdefault(child.tag, {}).update(child.attrib)

    def attrs(self, tag: str, el: ET.Element, childclass: str) -> Dict[str, str]:
        cls = el.get("class", childclass)
        base = dict(self.classes[cls].get(tag, self.classes["main"].get(tag, {})))
        base.update({k: v for k, v in el.attrib.items() if k != "class"})
        return base


# --------------------------------------------------------------------------------------
# the compiled model
# --------------------------------------------------------------------------------------

@dataclass
class Model:
    name: str
    arrays: Dict[str, np.ndarray] = field(default_factory=dict)
    names: Dict[str, List[str]] = field(default_factory=dict)
    hulls: List[Hull] = field(default_factory=list)

    def __getattr__(self, k):
        arrays = self.__dict__.get("arrays", {})
        if k in arrays:
            v = arrays[k]
            return int(v) if v.ndim == 0 and v.dtype.kind in "iu" else (float(v) if v.ndim == 0 else v)
        raise AttributeError(k)

    def id(self, kind: str, name: str) -> int:
        return self.names[kind].index(name)

    # ---- (de)serialisation: npz with allow_pickle=False compatible content ----
    def save(self, path: str):
        out = {f"a_{k}": v for k, v in self.arrays.items()}
        for k, v in self.names.items():
            out[f"n_{k}"] = np.array(v, dtype=np.str_)
        for i, h in enumerate(self.hulls):
            out[f"h{i}_vert"] = h.vert
            out[f"h{i}_fnormal"] = h.face_normal
            out[f"h{i}_foffset"] = h.face_offset
            out[f"h{i}_edge"] = h.edge
            fv = np.full((len(h.face_vert), max(len(f) for f in h.face_vert)), -1, dtype=np.int64)
            for j, f in enumerate(h.face_vert):
                fv[j, :len(f)] = f
            out[f"h{i}_fvert"] = fv
        out["model_name"] = np.array(self.name)
        np.savez_compressed(path, **out)

    @staticmethod
    def load(path: str) -> "Model":
        z = np.load(path, allow_pickle=False)
        m = Model(name=str(z["model_name"]))
        nh = 0
        for k in z.files:
            if k.startswith("a_"):
                m.arrays[k[2:]] = z[k]
            elif k.startswith("n_"):
                m.names[k[2:]] = [str(s) for s in z[k]]
            elif k.startswith("h") and k.endswith("_vert"):
                nh = max(nh, int(k[1:].split("_")[0]) + 1)
        for i in range(nh):
            fv = z[f"h{i}_fvert"]
            m.hulls.append(Hull(vert=z[f"h{i}_vert"], face_normal=z[f"h{i}_fnormal"],
                                face_offset=z[f"h{i}_foffset"], edge=z[f"h{i}_edge"],
                                face_vert=[[int(v) for v in row if v >= 0] for row in fv]))
        return m


def compile_mjcf(path: str, timestep: Optional[float] = None, asset_dir: Optional[str] = None) -> Model:
    """Compile one scene file into a :class:`Model` (``asset_dir`` overrides the scene directory)."""
    root = _load_tree(path)
    base_dir = asset_dir or os.path.dirname(path)
    meshdir = base_dir
    for comp in root.iter("compiler"):
        if comp.get("meshdir"):
            meshdir = os.path.join(base_dir, comp.get("meshdir"))
        if comp.get("angle", "degree") != "radian":
            raise NotImplementedError("only angle='radian' scenes are supported")

    defaults = _Defaults()
    for d in root.findall("default"):
        defaults.parse(d, "main")

    # options
    opt = dict(timestep=0.002, gravity=np.array([0, 0, -9.81]), impratio=1.0, tolerance=1e-8,
               ls_tolerance=0.01, iterations=100, ls_iterations=50, eulerdamp=1)
    for o in root.findall("option"):
        if o.get("timestep"):
            opt["timestep"] = float(o.get("timestep"))
        if o.get("gravity"):
            opt["gravity"] = _vec(o.get("gravity"), 3)
        if o.get("impratio"):
            opt["impratio"] = float(o.get("impratio"))
        if o.get("iterations"):
            opt["iterations"] = int(o.get("iterations"))
        if o.get("ls_iterations"):
            opt["ls_iterations"] = int(o.get("ls_iterations"))
        if o.get("tolerance"):
            opt["tolerance"] = float(o.get("tolerance"))
        for fl in o.findall("flag"):
            if fl.get("eulerdamp"):
                opt["eulerdamp"] = 0 if fl.get("eulerdamp") == "disable" else 1
        if o.get("cone", "pyramidal") != "pyramidal" or o.get("solver", "Newton") != "Newton" \
                or o.get("integrator", "Euler") != "Euler":
            raise NotImplementedError("only pyramidal cone / Newton / Euler are supported")
    if timestep is not None:
        opt["timestep"] = timestep

    # assets
    mesh_files: Dict[str, str] = {}
    mesh_scale: Dict[str, np.ndarray] = {}
    hfields: Dict[str, Tuple[np.ndarray, np.ndarray]] = {}
    for asset in root.findall("asset"):
        for me in asset.findall("mesh"):
            f = me.get("file")
            nm = me.get("name", os.path.splitext(os.path.basename(f))[0])
            mesh_files[nm] = os.path.join(meshdir, f)
            mesh_scale[nm] = _vec(me.get("scale"), 3) if me.get("scale") else np.ones(3)  # mesh/@scale
        for hf in asset.findall("hfield"):
            nm = hf.get("name")
            data = read_hfield_png(os.path.join(base_dir, hf.get("file")))
            hfields[nm] = (data, _vec(hf.get("size"), 4))

    # ---------------- body tree ----------------
    bodies = [dict(name="world", parent=-1, pos=np.zeros(3), quat=np.array([1.0, 0, 0, 0]),
                   ipos=np.zeros(3), iquat=np.array([1.0, 0, 0, 0]), mass=0.0, inertia=np.zeros(3), joints=[])]
    joints, geoms, sites = [], [], []

    def walk(el: ET.Element, parent: int, childclass: str):
        for child in el:
            if child.tag != "body":
                continue
            cc = child.get("childclass", childclass)
            b = dict(name=child.get("name", f"body{len(bodies)}"), parent=parent,
                     pos=_vec(child.get("pos", "0 0 0"), 3), quat=quat_normalize(_vec(child.get("quat", "1 0 0 0"), 4)),
                     ipos=np.zeros(3), iquat=np.array([1.0, 0, 0, 0]), mass=0.0, inertia=np.zeros(3), joints=[])
            bid = len(bodies)
            bodies.append(b)
            for sub in child:
                if sub.tag == "inertial":
                    b["ipos"] = _vec(sub.get("pos", "0 0 0"), 3)
                    b["mass"] = float(sub.get("mass"))
                    if sub.get("fullinertia"):
                        fi = _vec(sub.get("fullinertia"), 6)
                        I = np.array([[fi[0], fi[3], fi[4]], [fi[3], fi[1], fi[5]], [fi[4], fi[5], fi[2]]])
                        w, V = np.linalg.eigh(I)
                        order = np.argsort(-w)  # MuJoCo orders principal moments decreasingly
                        w, V = w[order], V[:, order]
                        if np.linalg.det(V) < 0:
                            V[:, 2] = -V[:, 2]
                        b["inertia"] = w
                        b["iquat"] = mat2quat(V)
                    else:
                        b["inertia"] = _vec(sub.get("diaginertia"), 3)
                        b["iquat"] = quat_normalize(_vec(sub.get("quat", "1 0 0 0"), 4))
                elif sub.tag in ("joint", "freejoint"):
                    if sub.tag == "freejoint":
                        a = dict(_DEFAULT_JOINT)
                        a.update(sub.attrib)
                        a["type"] = "free"
                    else:
                        a = defaults.attrs("joint", sub, cc)
                    jtype = {"free": JNT_FREE, "ball": JNT_BALL, "slide": JNT_SLIDE, "hinge": JNT_HINGE}[a["type"]]
                    rng = _vec(a.get("range"), 2) if a.get("range") else None
                    lim = a.get("limited", "auto")
                    limited = (rng is not None) if lim == "auto" else (lim == "true")
                    axis = _vec(a.get("axis", "0 0 1"), 3)
                    joints.append(dict(name=a.get("name", f"joint{len(joints)}"), type=jtype, body=bid,
                                       pos=_vec(a.get("pos", "0 0 0"), 3), axis=axis / np.linalg.norm(axis),
                                       limited=int(limited and jtype in (JNT_SLIDE, JNT_HINGE)),
                                       range=rng if rng is not None else np.zeros(2),
                                       damping=float(a.get("damping", 0)),
                                       frictionloss=float(a.get("frictionloss", 0)),
                                       armature=float(a.get("armature", 0)), margin=float(a.get("margin", 0)),
                                       solref=_vec(a.get("solreflimit", "0.02 1"), 2),
                                       solimp=_vec(a.get("solimplimit", "0.9 0.95 0.001 0.5 2"), 5),
                                       solreffriction=_vec(a.get("solreffriction", "0.02 1"), 2),
                                       solimpfriction=_vec(a.get("solimpfriction", "0.9 0.95 0.001 0.5 2"), 5)))
                    b["joints"].append(len(joints) - 1)
                elif sub.tag == "geom":
                    a = defaults.attrs("geom", sub, cc)
                    gtype = GEOM_TYPES[a.get("type", "sphere")]
                    geoms.append(dict(name=a.get("name", ""), type=gtype, body=bid, pos=_vec(a.get("pos"), 3),
                                      quat=quat_normalize(_vec(a.get("quat", "1 0 0 0"), 4)),
                                      contype=int(a.get("contype")), conaffinity=int(a.get("conaffinity")),
                                      condim=int(a.get("condim")), priority=int(a.get("priority")),
                                      friction=_merge_friction(a.get("friction")),
                                      solref=_vec(a.get("solref"), 2), solimp=_vec(a.get("solimp"), 5),
                                      margin=float(a.get("margin")), gap=float(a.get("gap")),
                                      solmix=float(a.get("solmix", 1)),
                                      size=np.pad(_vec(a.get("size")), (0, 3))[:3], mesh=a.get("mesh"),
                                      hfield=a.get("hfield"), group=int(a.get("group", 0))))
                elif sub.tag == "site":
                    a = defaults.attrs("site", sub, cc)
                    sites.append(dict(name=a.get("name", f"site{len(sites)}"), body=bid, pos=_vec(a.get("pos"), 3),
                                      quat=quat_normalize(_vec(a.get("quat", "1 0 0 0"), 4))))
            walk(child, bid, cc)

    for wb in root.findall("worldbody"):
        for sub in wb:
            if sub.tag == "geom":
                a = defaults.attrs("geom", sub, "main")
                geoms_world = dict(name=a.get("name", ""), type=GEOM_TYPES[a.get("type", "sphere")], body=0,
                                   pos=_vec(a.get("pos"), 3), quat=quat_normalize(_vec(a.get("quat", "1 0 0 0"), 4)),
                                   contype=int(a.get("contype")), conaffinity=int(a.get("conaffinity")),
                                   condim=int(a.get("condim")), priority=int(a.get("priority")),
                                   friction=_merge_friction(a.get("friction")), solref=_vec(a.get("solref"), 2),
                                   solimp=_vec(a.get("solimp"), 5), margin=float(a.get("margin")),
                                   gap=float(a.get("gap")), solmix=float(a.get("solmix", 1)),
                                   size=np.pad(_vec(a.get("size")), (0, 3))[:3], mesh=a.get("mesh"),
                                   hfield=a.get("hfield"), group=int(a.get("group", 0)))
                geoms.append(geoms_world)
        walk(wb, 0, "main")

    # MuJoCo orders geoms by body (depth-first body order, then XML order within a body)
    geoms = sorted(enumerate(geoms), key=lambda ig: (ig[1]["body"], ig[0]))
    geoms = [g for _, g in geoms]
    sites = sorted(enumerate(sites), key=lambda s: (s[1]["body"], s[0]))
    sites = [s for _, s in sites]

    nbody = len(bodies)
    njnt = len(joints)

    # ---------------- addresses ----------------
    jnt_qposadr, jnt_dofadr = [], []
    nq = nv = 0
    dof_body, dof_jnt = [], []
    for j in joints:
        jnt_qposadr.append(nq)
        jnt_dofadr.append(nv)
        nqj, nvj = {JNT_FREE: (7, 6), JNT_BALL: (4, 3), JNT_SLIDE: (1, 1), JNT_HINGE: (1, 1)}[j["type"]]
        nq += nqj
        nv += nvj
        for _ in range(nvj):
            dof_body.append(j["body"])
            dof_jnt.append(len(dof_jnt) and 0)  # placeholder
    dof_jnt = []
    for ji, j in enumerate(joints):
        nvj = {JNT_FREE: 6, JNT_BALL: 3, JNT_SLIDE: 1, JNT_HINGE: 1}[j["type"]]
        dof_jnt += [ji] * nvj

    body_parent = np.array([b["parent"] for b in bodies], dtype=np.int64)
    body_jntnum = np.array([len(b["joints"]) for b in bodies], dtype=np.int64)
    body_jntadr = np.array([b["joints"][0] if b["joints"] else -1 for b in bodies], dtype=np.int64)
    body_dofnum = np.zeros(nbody, dtype=np.int64)
    body_dofadr = -np.ones(nbody, dtype=np.int64)
    for d, b in enumerate(dof_body):
        if body_dofadr[b] < 0:
            body_dofadr[b] = d
        body_dofnum[b] += 1
    body_rootid = np.zeros(nbody, dtype=np.int64)
    body_weldid = np.zeros(nbody, dtype=np.int64)
    for i in range(1, nbody):
        p = body_parent[i]
        body_rootid[i] = i if p == 0 else body_rootid[p]
        body_weldid[i] = i if body_jntnum[i] > 0 else body_weldid[p]
    # dof parent: previous dof in the same body, else last dof of the nearest ancestor with dofs
    dof_parent = -np.ones(nv, dtype=np.int64)
    for d in range(nv):
        b = dof_body[d]
        if d > 0 and dof_body[d - 1] == b:
            dof_parent[d] = d - 1
        else:
            p = body_parent[b]
            while p > 0 and body_dofnum[p] == 0:
                p = body_parent[p]
            dof_parent[d] = body_dofadr[p] + body_dofnum[p] - 1 if p > 0 else -1

    # qpos0
    qpos0 = np.zeros(nq)
    for ji, j in enumerate(joints):
        a = jnt_qposadr[ji]
        if j["type"] == JNT_FREE:
            qpos0[a:a + 3] = bodies[j["body"]]["pos"]
            qpos0[a + 3:a + 7] = bodies[j["body"]]["quat"]
        elif j["type"] == JNT_BALL:
            qpos0[a:a + 4] = [1, 0, 0, 0]

    # ---------------- actuators ----------------
    acts = []
    for actsec in root.findall("actuator"):
        for a_el in actsec:
            if a_el.tag != "position":
                raise NotImplementedError(f"actuator type {a_el.tag}")
            a = defaults.attrs("position", a_el, "main")
            jid = [j["name"] for j in joints].index(a["joint"])
            kp, kv = float(a.get("kp", 1)), float(a.get("kv", 0))
            ctrlrange = _vec(a.get("ctrlrange"), 2) if a.get("ctrlrange") else None
            inherit = float(a.get("inheritrange", 0))
            if inherit > 0:
                lo, hi = joints[jid]["range"]
                c, r = (lo + hi) / 2, (hi - lo) / 2 * inherit
                ctrlrange = np.array([c - r, c + r])
            forcerange = _vec(a.get("forcerange"), 2) if a.get("forcerange") else None
            cl, fl = a.get("ctrllimited", "auto"), a.get("forcelimited", "auto")
            acts.append(dict(name=a.get("name"), joint=jid, kp=kp, kv=kv, gear=float(a.get("gear", 1)),
                             ctrllimited=int((ctrlrange is not None) if cl == "auto" else cl == "true"),
                             forcelimited=int((forcerange is not None) if fl == "auto" else fl == "true"),
                             ctrlrange=ctrlrange if ctrlrange is not None else np.zeros(2),
                             forcerange=forcerange if forcerange is not None else np.zeros(2)))
    nu = len(acts)

    # ---------------- sensors ----------------
    sens = []
    adr = 0
    site_names = [s["name"] for s in sites]
    for ss in root.findall("sensor"):
        for s_el in ss:
            typ, dim = SENSOR_TYPES[s_el.tag]
            obj = s_el.get("site") or s_el.get("objname")
            if s_el.get("objtype", "site") != "site":
                raise NotImplementedError("only site sensors")
            sens.append(dict(name=s_el.get("name"), type=typ, objid=site_names.index(obj), adr=adr, dim=dim))
            adr += dim
    nsensordata = adr

    # ---------------- keyframe ----------------
    key_qpos, key_ctrl, key_names = [], [], []
    for kf in root.findall("keyframe"):
        for k in kf.findall("key"):
            key_names.append(k.get("name"))
            key_qpos.append(_vec(k.get("qpos"), nq) if k.get("qpos") else qpos0.copy())
            key_ctrl.append(_vec(k.get("ctrl"), nu) if k.get("ctrl") else np.zeros(nu))

    # ---------------- collision geometry ----------------
    hulls: List[Hull] = []
    mesh_hull_id: Dict[str, int] = {}
    geom_dataid = []
    geom_rbound = []
    for g in geoms:
        if g["type"] == GEOM_MESH and (g["contype"] or g["conaffinity"]):
            if g["mesh"] not in mesh_hull_id:
                hulls.append(convex_hull(read_stl(mesh_files[g["mesh"]]) * mesh_scale[g["mesh"]]))
                mesh_hull_id[g["mesh"]] = len(hulls) - 1
            hid = mesh_hull_id[g["mesh"]]
            geom_dataid.append(hid)
            geom_rbound.append(float(np.max(np.linalg.norm(hulls[hid].vert, axis=1))))
        elif g["type"] == GEOM_HFIELD:
            geom_dataid.append(list(hfields).index(g["hfield"]))
            geom_rbound.append(0.0)
        else:
            geom_dataid.append(-1)
            geom_rbound.append(0.0)

    def is_ancestor_weld(b1, b2):
        # MuJoCo filterparent: exclude body pairs where one weld-body is the parent of the other
        w1, w2 = body_weldid[b1], body_weldid[b2]
        return w1 == w2 or body_weldid[body_parent[w1]] == w2 or body_weldid[body_parent[w2]] == w1

    pairs = []
    for i in range(len(geoms)):
        for j in range(i + 1, len(geoms)):
            g1, g2 = geoms[i], geoms[j]
            if not ((g1["contype"] & g2["conaffinity"]) or (g2["contype"] & g1["conaffinity"])):
                continue
            b1, b2 = g1["body"], g2["body"]
            if body_weldid[b1] == body_weldid[b2]:
                continue
            if body_weldid[b1] != 0 and body_weldid[b2] != 0 and is_ancestor_weld(b1, b2):
                continue
            if body_weldid[b1] == 0 and body_weldid[b2] == 0:
                continue
            # order by geom type (lower type first, MuJoCo convention), keep ids
            if g1["type"] > g2["type"]:
                i1, i2 = j, i
            else:
                i1, i2 = i, j
            ga, gb = geoms[i1], geoms[i2]
            if ga["priority"] != gb["priority"]:
                w = ga if ga["priority"] > gb["priority"] else gb
                condim, fr, solref, solimp = w["condim"], w["friction"], w["solref"], w["solimp"]
            else:
                condim = max(ga["condim"], gb["condim"])
                fr = np.maximum(ga["friction"], gb["friction"])
                mix = 0.5 if ga["solmix"] + gb["solmix"] <= 0 else ga["solmix"] / (ga["solmix"] + gb["solmix"])
                solref = mix * ga["solref"] + (1 - mix) * gb["solref"]
                solimp = mix * ga["solimp"] + (1 - mix) * gb["solimp"]
            pairs.append(dict(g1=i1, g2=i2, condim=condim,
                              friction=np.array([fr[0], fr[0], fr[1], fr[2], fr[2]]),
                              solref=solref, solimp=solimp, margin=max(ga["margin"], gb["margin"]),
                              gap=max(ga["gap"], gb["gap"])))

    A: Dict[str, np.ndarray] = {}
    I = lambda x: np.asarray(x, dtype=np.int64)
    F = lambda x: np.asarray(x, dtype=np.float64)
    A.update(nq=I(nq), nv=I(nv), nu=I(nu), nbody=I(nbody), njnt=I(njnt), ngeom=I(len(geoms)), nsite=I(len(sites)),
             nsensor=I(len(sens)), nsensordata=I(nsensordata), npair=I(len(pairs)), nkey=I(len(key_names)))
    A["opt_timestep"] = F(opt["timestep"])
    A["opt_gravity"] = F(opt["gravity"])
    A["opt_impratio"] = F(opt["impratio"])
    A["opt_tolerance"] = F(opt["tolerance"])
    A["opt_ls_tolerance"] = F(opt["ls_tolerance"])
    A["opt_iterations"] = I(opt["iterations"])
    A["opt_ls_iterations"] = I(opt["ls_iterations"])
    A["opt_eulerdamp"] = I(opt["eulerdamp"])
    A["body_parentid"] = body_parent
    A["body_rootid"] = body_rootid
    A["body_weldid"] = body_weldid
    A["body_jntnum"] = body_jntnum
    A["body_jntadr"] = body_jntadr
    A["body_dofnum"] = body_dofnum
    A["body_dofadr"] = body_dofadr
    A["body_pos"] = F([b["pos"] for b in bodies])
    A["body_quat"] = F([b["quat"] for b in bodies])
    A["body_ipos"] = F([b["ipos"] for b in bodies])
    A["body_iquat"] = F([b["iquat"] for b in bodies])
    A["body_mass"] = F([b["mass"] for b in bodies])
    A["body_inertia"] = F([b["inertia"] for b in bodies])
    A["jnt_type"] = I([j["type"] for j in joints])
    A["jnt_qposadr"] = I(jnt_qposadr)
    A["jnt_dofadr"] = I(jnt_dofadr)
    A["jnt_bodyid"] = I([j["body"] for j in joints])
    A["jnt_pos"] = F([j["pos"] for j in joints])
    A["jnt_axis"] = F([j["axis"] for j in joints])
    A["jnt_limited"] = I([j["limited"] for j in joints])
    A["jnt_range"] = F([j["range"] for j in joints])
    A["jnt_margin"] = F([j["margin"] for j in joints])
    A["jnt_solref"] = F([j["solref"] for j in joints])
    A["jnt_solimp"] = F([j["solimp"] for j in joints])
    A["dof_bodyid"] = I(dof_body)
    A["dof_jntid"] = I(dof_jnt)
    A["dof_parentid"] = dof_parent
    A["dof_armature"] = F([joints[j]["armature"] for j in dof_jnt])
    A["dof_damping"] = F([joints[j]["damping"] for j in dof_jnt])
    A["dof_frictionloss"] = F([joints[j]["frictionloss"] for j in dof_jnt])
    A["dof_solref"] = F([joints[j]["solreffriction"] for j in dof_jnt])
    A["dof_solimp"] = F([joints[j]["solimpfriction"] for j in dof_jnt])
    A["geom_type"] = I([g["type"] for g in geoms])
    A["geom_bodyid"] = I([g["body"] for g in geoms])
    A["geom_pos"] = F([g["pos"] for g in geoms])
    A["geom_quat"] = F([g["quat"] for g in geoms])
    A["geom_contype"] = I([g["contype"] for g in geoms])
    A["geom_conaffinity"] = I([g["conaffinity"] for g in geoms])
    A["geom_condim"] = I([g["condim"] for g in geoms])
    A["geom_priority"] = I([g["priority"] for g in geoms])
    A["geom_friction"] = F([g["friction"] for g in geoms])
    A["geom_size"] = F([g["size"] for g in geoms])
    A["geom_dataid"] = I(geom_dataid)
    A["geom_rbound"] = F(geom_rbound)
    A["site_bodyid"] = I([s["body"] for s in sites])
    A["site_pos"] = F([s["pos"] for s in sites])
    A["site_quat"] = F([s["quat"] for s in sites])
    A["actuator_trnid"] = I([a["joint"] for a in acts])
    A["actuator_gear"] = F([a["gear"] for a in acts])
    A["actuator_kp"] = F([a["kp"] for a in acts])
    A["actuator_kv"] = F([a["kv"] for a in acts])
    A["actuator_ctrllimited"] = I([a["ctrllimited"] for a in acts])
    A["actuator_forcelimited"] = I([a["forcelimited"] for a in acts])
    A["actuator_ctrlrange"] = F([a["ctrlrange"] for a in acts])
    A["actuator_forcerange"] = F([a["forcerange"] for a in acts])
    # gain/bias parameters as MuJoCo stores them for <position>
    gp = np.zeros((nu, 10))
    bp = np.zeros((nu, 10))
    for i, a in enumerate(acts):
        gp[i, 0] = a["kp"]
        bp[i, 1] = -a["kp"]
        bp[i, 2] = -a["kv"]
    A["actuator_gainprm"] = gp
    A["actuator_biasprm"] = bp
    A["sensor_type"] = I([s["type"] for s in sens])
    A["sensor_objid"] = I([s["objid"] for s in sens])
    A["sensor_adr"] = I([s["adr"] for s in sens])
    A["sensor_dim"] = I([s["dim"] for s in sens])
    A["key_qpos"] = F(key_qpos).reshape(len(key_names), nq)
    A["key_ctrl"] = F(key_ctrl).reshape(len(key_names), nu)
    A["qpos0"] = qpos0
    A["pair_geom1"] = I([p["g1"] for p in pairs])
    A["pair_geom2"] = I([p["g2"] for p in pairs])
    A["pair_condim"] = I([p["condim"] for p in pairs])
    A["pair_friction"] = F([p["friction"] for p in pairs]).reshape(len(pairs), 5)
    A["pair_solref"] = F([p["solref"] for p in pairs]).reshape(len(pairs), 2)
    A["pair_solimp"] = F([p["solimp"] for p in pairs]).reshape(len(pairs), 5)
    A["pair_margin"] = F([p["margin"] for p in pairs])
    A["pair_gap"] = F([p["gap"] for p in pairs])
    if hfields:
        (hdata, hsize), = list(hfields.values())
        A["hfield_size"] = F(hsize)
        A["hfield_nrow"] = I(hdata.shape[0])
        A["hfield_ncol"] = I(hdata.shape[1])
        A["hfield_data"] = F(hdata)
    else:
        A["hfield_nrow"] = I(0)
        A["hfield_ncol"] = I(0)
        A["hfield_size"] = F(np.zeros(4))
        A["hfield_data"] = F(np.zeros((0, 0)))

    names = dict(body=[b["name"] for b in bodies], jnt=[j["name"] for j in joints], geom=[g["name"] for g in geoms],
                 site=[s["name"] for s in sites], actuator=[a["name"] for a in acts],
                 sensor=[s["name"] for s in sens], key=key_names)
    model = Model(name=os.path.basename(path), arrays=A, names=names, hulls=hulls)
    set_const(model)
    return model


def _merge_friction(s: str) -> np.ndarray:
    out = np.array([1.0, 0.005, 0.0001])
    v = _vec(s)
    out[:v.size] = v
    return out


# --------------------------------------------------------------------------------------
# mj_setConst-style constants computed at qpos0 (numpy, fp64)
# --------------------------------------------------------------------------------------

def _kinematics_np(m: Model, qpos: np.ndarray):
    nb = m.nbody
    xpos = np.zeros((nb, 3))
    xquat = np.zeros((nb, 4))
    xquat[0] = [1, 0, 0, 0]
    xanchor = np.zeros((m.njnt, 3))
    xaxis = np.zeros((m.njnt, 3))
    for i in range(1, nb):
        p = m.body_parentid[i]
        ja, jn = m.body_jntadr[i], m.body_jntnum[i]
        if jn and m.jnt_type[ja] == JNT_FREE:
            a = m.jnt_qposadr[ja]
            xpos[i] = qpos[a:a + 3]
            xquat[i] = quat_normalize(qpos[a + 3:a + 7])
            xanchor[ja] = xpos[i]
            xaxis[ja] = [0, 0, 1]
            continue
        xpos[i] = xpos[p] + quat2mat(xquat[p]) @ m.body_pos[i]
        q = quat_mul(xquat[p], m.body_quat[i])
        for j in range(ja, ja + jn):
            R = quat2mat(q)
            xanchor[j] = R @ m.jnt_pos[j] + xpos[i]
            xaxis[j] = R @ m.jnt_axis[j]
            a = m.jnt_qposadr[j]
            if m.jnt_type[j] == JNT_HINGE:
                q = quat_mul(q, axis_angle_quat(m.jnt_axis[j], qpos[a] - m.qpos0[a]))
                xpos[i] = xanchor[j] - quat2mat(q) @ m.jnt_pos[j]
            else:
                raise NotImplementedError
        xquat[i] = quat_normalize(q)
    xmat = np.array([quat2mat(q) for q in xquat])
    xipos = np.array([xpos[i] + xmat[i] @ m.body_ipos[i] for i in range(nb)])
    ximat = np.array([xmat[i] @ quat2mat(m.body_iquat[i]) for i in range(nb)])
    return xpos, xmat, xipos, ximat, xanchor, xaxis


def mass_matrix_np(m: Model, qpos: np.ndarray):
    """Dense M(q) via composite rigid bodies in MuJoCo's com-based spatial algebra (fp64)."""
    nb, nv = m.nbody, m.nv
    xpos, xmat, xipos, ximat, xanchor, xaxis = _kinematics_np(m, qpos)
    # subtree com of each root
    mass = m.body_mass
    subtree_com = np.zeros((nb, 3))
    subtree_mass = mass.copy()
    acc = xipos * mass[:, None]
    for i in range(nb - 1, 0, -1):
        p = m.body_parentid[i]
        acc[p] += acc[i]
        subtree_mass[p] += subtree_mass[i]
    for i in range(nb):
        subtree_com[i] = acc[i] / subtree_mass[i] if subtree_mass[i] > MJMINVAL else xipos[i]
    cinert = np.zeros((nb, 6, 6))
    for i in range(1, nb):
        c = subtree_com[m.body_rootid[i]]
        d = xipos[i] - c
        Ib = ximat[i] @ np.diag(m.body_inertia[i]) @ ximat[i].T
        Ib += mass[i] * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
        h = mass[i] * d
        S = np.array([[0, -h[2], h[1]], [h[2], 0, -h[0]], [-h[1], h[0], 0]])
        cinert[i][:3, :3] = Ib
        cinert[i][:3, 3:] = S
        cinert[i][3:, :3] = -S
        cinert[i][3:, 3:] = mass[i] * np.eye(3)
    cdof = np.zeros((nv, 6))
    for j in range(m.njnt):
        b = m.jnt_bodyid[j]
        c = subtree_com[m.body_rootid[b]]
        da = m.jnt_dofadr[j]
        if m.jnt_type[j] == JNT_FREE:
            for k in range(3):
                cdof[da + k, 3 + k] = 1
            for k in range(3):
                ax = xmat[b][:, k]
                cdof[da + 3 + k, :3] = ax
                cdof[da + 3 + k, 3:] = np.cross(ax, c - xanchor[j])
        else:
            ax = xaxis[j]
            cdof[da, :3] = ax
            cdof[da, 3:] = np.cross(ax, c - xanchor[j])
    crb = cinert.copy()
    for i in range(nb - 1, 0, -1):
        p = m.body_parentid[i]
        if p > 0:
            crb[p] += crb[i]
    M = np.zeros((nv, nv))
    for i in range(nv):
        f = crb[m.dof_bodyid[i]] @ cdof[i]
        j = i
        while j >= 0:
            M[i, j] = M[j, i] = cdof[j] @ f
            j = m.dof_parentid[j]
        M[i, i] += m.dof_armature[i]
    return M, dict(xpos=xpos, xmat=xmat, xipos=xipos, ximat=ximat, cdof=cdof, subtree_com=subtree_com,
                   subtree_mass=subtree_mass)


def set_const(m: Model):
    M, kin = mass_matrix_np(m, m.qpos0)
    Minv = np.linalg.inv(M)
    nv = m.nv
    diag = np.diag(Minv)
    dof_iw = np.zeros(nv)
    for j in range(m.njnt):
        da = m.jnt_dofadr[j]
        if m.jnt_type[j] == JNT_FREE:
            dof_iw[da:da + 3] = diag[da:da + 3].mean()
            dof_iw[da + 3:da + 6] = diag[da + 3:da + 6].mean()
        elif m.jnt_type[j] == JNT_BALL:
            dof_iw[da:da + 3] = diag[da:da + 3].mean()
        else:
            dof_iw[da] = diag[da]
    body_iw = np.zeros((m.nbody, 2))
    for b in range(1, m.nbody):
        if m.body_weldid[b] == 0:
            continue
        c = kin["subtree_com"][m.body_rootid[b]]
        p = kin["xipos"][b]
        J = np.zeros((6, nv))
        d = m.body_dofadr[m.body_weldid[b]] + m.body_dofnum[m.body_weldid[b]] - 1
        while d >= 0:
            cd = kin["cdof"][d]
            J[:3, d] = cd[3:] + np.cross(cd[:3], p - c)
            J[3:, d] = cd[:3]
            d = m.dof_parentid[d]
        A6 = J @ Minv @ J.T
        body_iw[b, 0] = max(MJMINVAL, np.trace(A6[:3, :3]) / 3)
        body_iw[b, 1] = max(MJMINVAL, np.trace(A6[3:, 3:]) / 3)
    m.arrays["dof_invweight0"] = dof_iw
    m.arrays["body_invweight0"] = body_iw
    m.arrays["stat_meaninertia"] = np.asarray(np.trace(M) / nv)
    m.arrays["body_subtreemass"] = kin["subtree_mass"]
    m.arrays["qM0"] = M
