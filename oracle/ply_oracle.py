"""TEST INFRASTRUCTURE -- CPU restatement of the reference's PLY loader, for checking the
native reader (gaussiansplattingviewer_amd/csrc/ply_loader.hip).  Never imported by the
product path.

`load_ply_reference` follows util_gau.load_ply (reference util_gau.py:63-125) statement by
statement, in numpy, on the property arrays that `read_vertex` returns.  `read_vertex` stands
in for plyfile (absent here): it reads the vertex element of a binary
little / big endian or ascii PLY into one numpy array per property, with the property's own
dtype as plyfile does (ascii values are parsed as float64 and cast, like plyfile's text path).
`write_ply` writes the 3D Gaussian Splatting layout for fixtures.
"""
from __future__ import annotations

import numpy as np

_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2",
          "int16": "i2", "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4",
          "uint": "u4", "uint32": "u4", "float": "f4", "float32": "f4", "double": "f8",
          "float64": "f8"}


def read_vertex(path):
    """{property name: 1-D array} of the vertex element (plyfile's elements[0][name])."""
    with open(path, "rb") as f:
        data = f.read()
    end = data.index(b"end_header") + len(b"end_header")
    end = data.index(b"\n", end) + 1
    header = data[:end].decode("ascii").splitlines()
    fmt, props, count, in_vertex = None, [], 0, False
    for line in header:
        w = line.split()
        if not w:
            continue
        if w[0] == "format":
            fmt = w[1]
        elif w[0] == "element":
            in_vertex = w[1] == "vertex"
            if in_vertex:
                count = int(w[2])
        elif w[0] == "property" and in_vertex:
            props.append((w[2], _TYPES[w[1]]))
    if fmt == "ascii":
        vals = np.array(data[end:].split()[:count * len(props)], dtype=np.float64)
        vals = vals.reshape(count, len(props))
        return {n: vals[:, i].astype(t) for i, (n, t) in enumerate(props)}
    order = "<" if fmt == "binary_little_endian" else ">"
    dt = np.dtype([(n, order + t) for n, t in props])
    arr = np.frombuffer(data, dtype=dt, count=count, offset=end)
    return {n: arr[n].astype(np.dtype(t)) for n, t in props}


def load_ply_reference(path):
    """util_gau.load_ply restated: (xyz, rot, scale, opacity, sh, bounding_box, center)."""
    max_sh_degree = 3
    el = read_vertex(path)
    names = list(el)
    xyz = np.stack((np.asarray(el["x"]), np.asarray(el["y"]), np.asarray(el["z"])), axis=1)
    opacities = np.asarray(el["opacity"])[..., np.newaxis]
    min_bound = xyz.min(axis=0)
    max_bound = xyz.max(axis=0)
    bounding_box = np.array([min_bound, max_bound])
    center = xyz.mean(axis=0)
    features_dc = np.zeros((xyz.shape[0], 3, 1))
    features_dc[:, 0, 0] = np.asarray(el["f_dc_0"])
    features_dc[:, 1, 0] = np.asarray(el["f_dc_1"])
    features_dc[:, 2, 0] = np.asarray(el["f_dc_2"])
    extra_f_names = [p for p in names if p.startswith("f_rest_")]
    extra_f_names = sorted(extra_f_names, key=lambda x: int(x.split('_')[-1]))
    assert len(extra_f_names) == 3 * (max_sh_degree + 1) ** 2 - 3
    features_extra = np.zeros((xyz.shape[0], len(extra_f_names)))
    for idx, attr_name in enumerate(extra_f_names):
        features_extra[:, idx] = np.asarray(el[attr_name])
    features_extra = features_extra.reshape((features_extra.shape[0], 3, (max_sh_degree + 1) ** 2 - 1))
    features_extra = np.transpose(features_extra, [0, 2, 1])
    scale_names = sorted([p for p in names if p.startswith("scale_")], key=lambda x: int(x.split('_')[-1]))
    scales = np.zeros((xyz.shape[0], len(scale_names)))
    for idx, attr_name in enumerate(scale_names):
        scales[:, idx] = np.asarray(el[attr_name])
    rot_names = sorted([p for p in names if p.startswith("rot")], key=lambda x: int(x.split('_')[-1]))
    rots = np.zeros((xyz.shape[0], len(rot_names)))
    for idx, attr_name in enumerate(rot_names):
        rots[:, idx] = np.asarray(el[attr_name])
    xyz = xyz.astype(np.float32)
    rots = rots / np.linalg.norm(rots, axis=-1, keepdims=True)
    rots = rots.astype(np.float32)
    scales = np.exp(scales)
    scales = scales.astype(np.float32)
    opacities = 1 / (1 + np.exp(- opacities))
    opacities = opacities.astype(np.float32)
    shs = np.concatenate([features_dc.reshape(-1, 3),
                          features_extra.reshape(len(features_dc), -1)], axis=-1).astype(np.float32)
    return xyz, rots, scales, opacities, shs, bounding_box, center


GS_PROPS = (["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"]
            + [f"f_rest_{i}" for i in range(45)] + ["opacity", "scale_0", "scale_1", "scale_2",
                                                   "rot_0", "rot_1", "rot_2", "rot_3"])


def write_ply(path, values: dict, fmt="binary_little_endian", types=None, order=None):
    """Write a vertex-only PLY.  values: {name: 1-D array}; types: {name: PLY type} (default
    float); order: property order (default GS_PROPS filtered to the given names)."""
    names = order or [n for n in GS_PROPS if n in values] + [n for n in values if n not in GS_PROPS]
    types = types or {}
    P = len(values[names[0]])
    inv = {"i1": "char", "u1": "uchar", "i2": "short", "u2": "ushort", "i4": "int", "u4": "uint",
           "f4": "float", "f8": "double"}
    code = {n: np.dtype(_TYPES[types.get(n, "float")]).str[1:] for n in names}
    lines = ["ply", f"format {fmt} 1.0", "comment written by oracle/ply_oracle.py",
             f"element vertex {P}"] + [f"property {inv[code[n]]} {n}" for n in names] + ["end_header"]
    head = ("\n".join(lines) + "\n").encode("ascii")
    if fmt == "ascii":
        rows = []
        for i in range(P):
            rows.append(" ".join(repr(float(np.asarray(values[n][i]).astype(code[n]))) if code[n][0] == "f"
                                 else str(int(values[n][i])) for n in names))
        body = ("\n".join(rows) + "\n").encode("ascii")
    else:
        o = "<" if fmt == "binary_little_endian" else ">"
        arr = np.empty(P, dtype=[(n, o + code[n]) for n in names])
        for n in names:
            arr[n] = values[n]
        body = arr.tobytes()
    with open(path, "wb") as f:
        f.write(head + body)
