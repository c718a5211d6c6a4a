"""Mesh export (nerf/mesh.py, the reference's renderer.py:121-299 without
mcubes / xatlas / nvdiffrast): marching tetrahedra on analytic level sets.
The reference's own mesh library is absent, so these are properties of a
correct isosurface rather than a comparison with PyMCubes (parity unpinned):
vertices on the level set, a closed consistently oriented 2-manifold with
the right Euler characteristic, outward normals, nothing for a constant
field; plus the OBJ writer and the GPU export path."""
import numpy as np
import pytest
import torch

from nerf.mesh import isosurface, write_obj


def _lattice(n, lo=-1.0, hi=1.0):
    ax = np.linspace(lo, hi, n)
    return np.stack(np.meshgrid(ax, ax, ax, indexing="ij"), -1), (hi - lo) / (n - 1)


def _check_closed_oriented(faces):
    """Every directed edge once and its reverse once: a closed, consistently
    oriented 2-manifold.  Returns the undirected edge count."""
    d = np.concatenate([faces[:, [0, 1]], faces[:, [1, 2]], faces[:, [2, 0]]])
    key = d[:, 0].astype(np.int64) * (faces.max() + 1) + d[:, 1]
    rev = d[:, 1].astype(np.int64) * (faces.max() + 1) + d[:, 0]
    assert len(np.unique(key)) == len(key), "a directed edge repeats (orientation)"
    assert np.array_equal(np.sort(key), np.sort(rev)), "an edge is not shared by two faces"
    return len(key) // 2


def test_sphere_level_set():
    x, h = _lattice(40)
    r0 = 0.6
    vals = r0 - np.linalg.norm(x, axis=-1)  # > 0 inside
    verts, faces = isosurface(vals, 0.0)
    assert len(faces) > 1000
    pos = verts * h - 1.0
    r = np.linalg.norm(pos, axis=1)
    # linear interpolation of |x| along a lattice edge: error <= h^2 / (2 r)
    assert np.abs(r - r0).max() <= h * h / r0
    E = _check_closed_oriented(faces)
    assert len(verts) - E + len(faces) == 2  # a sphere
    p = pos[faces]
    nrm = np.cross(p[:, 1] - p[:, 0], p[:, 2] - p[:, 0])
    assert np.all((nrm * p.mean(1)).sum(1) > 0), "normals must point outward"


def test_torus_euler_characteristic_and_threshold():
    x, h = _lattice(48)
    R, rr = 0.55, 0.22
    q = np.sqrt(x[..., 0] ** 2 + x[..., 1] ** 2) - R
    dens = np.exp(-(q ** 2 + x[..., 2] ** 2) / (2 * 0.15 ** 2)) * 20.0  # a density blob
    thresh = 20.0 * np.exp(-rr ** 2 / (2 * 0.15 ** 2))
    verts, faces = isosurface(dens, thresh)
    E = _check_closed_oriented(faces)
    assert len(verts) - E + len(faces) == 0  # a torus
    # vertices interpolate the lattice values to the threshold exactly on the edge
    pos = verts * h - 1.0
    q = np.sqrt(pos[:, 0] ** 2 + pos[:, 1] ** 2) - R
    assert np.abs(np.sqrt(q ** 2 + pos[:, 2] ** 2) - rr).max() < 2 * h


def test_constant_and_degenerate_fields():
    for v in (np.zeros((8, 8, 8)), np.ones((8, 8, 8))):
        verts, faces = isosurface(v, 0.5)
        assert len(verts) == 0 and len(faces) == 0
    verts, faces = isosurface(np.ones((1, 4, 4)), 0.5)
    assert len(faces) == 0


def test_write_obj(tmp_path):
    x, h = _lattice(12)
    verts, faces = isosurface(0.5 - np.linalg.norm(x, axis=-1), 0.0)
    cols = np.full((len(verts), 3), 0.25)
    write_obj(tmp_path / "m.obj", verts, faces, cols)
    v, f = [], []
    for line in open(tmp_path / "m.obj"):
        t = line.split()
        if t and t[0] == "v":
            v.append([float(a) for a in t[1:]])
        elif t and t[0] == "f":
            f.append([int(a) - 1 for a in t[1:]])
    v, f = np.array(v), np.array(f)
    np.testing.assert_allclose(v[:, :3], verts, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(v[:, 3:], cols)
    assert np.array_equal(f, faces)


@pytest.mark.gpu
def test_export_mesh_on_gpu(gpu, tmp_path):
    """Trainer.save_mesh / NeRFRenderer.export_mesh after a few native
    training steps: the OBJ is written, lies in [-1, 1]^3 and is consistently
    oriented."""
    import bench
    trainer, data = bench.make_trainer(64, 3, 0, 1, True, graph=True)
    with torch.no_grad():
        trainer.model.encoder.embeddings.uniform_(-0.5, 0.5)
    for i in range(17):
        trainer.train_iteration(data.collate([i % 4]))
    trainer.workspace = str(tmp_path)
    trainer.log_ptr = None
    trainer.save_mesh(resolution=64)
    path = tmp_path / "mesh" / "mesh.obj"
    assert path.exists()
    verts, faces = trainer.model.export_mesh(str(tmp_path / "m2"), resolution=64)
    assert len(faces) > 0 and np.abs(verts).max() <= 1.0 + 1e-6
    # consistently oriented (a surface cut open by the lattice boundary is
    # allowed here: each directed edge appears at most once)
    f = faces.astype(np.int64)
    d = np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]])
    key = d[:, 0] * (f.max() + 1) + d[:, 1]
    assert len(np.unique(key)) == len(key)
