"""Mesh subtrees searched per lane in BVHs of their own (frt_engine.hip mesh_roots /
MeshBuild, frt_traverse.hpp MeshDesc).

CPU: the meshes frt_scene_upload would detect in each golden scene and their BVHs,
built by the same host code and checked by frt_mesh_check (every triangle of a mesh
in exactly one leaf, every box holding its triangles' vertices and its children's
boxes, every child's smallest pre-order index right). The GPU side — the search's
answer is the generic walk's, bit for bit — is test_gpu_parity.py
test_mesh_search_equals_generic_walk.
"""
import os

import pytest

from conftest import GOLDEN, load_scene

SCENES = sorted(f[:-2] for f in os.listdir(os.path.join(GOLDEN, "scenes")) if f.endswith(".c"))
# the scenes with meshes (groups of >= 64 triangles in trees over 512 nodes): meshes, triangles in them
# (bounding_boxes: 6 dragons of 23 490 faces each, dragon.obj)
MESHES = {"bounding_boxes_800x1000_4x4": (6, 140940), "bounding_boxes_100x125_4x4": (6, 140940),
          "bounding_boxes_200x80": (6, 140940), "degenerate_mesh_48": (1, 600)}


@pytest.mark.parametrize("name", SCENES)
def test_mesh_bvh_sound(built, name):
    from fast_ray_tracer_amd.runtime import mesh_check
    bad, st = mesh_check(load_scene(name))
    print(name, st)
    assert bad == 0, (name, bad, st)
    if name in MESHES:
        assert (st["meshes"], st["triangles"]) == MESHES[name], st
    if st["meshes"]:
        # a binary tree over T triangles in leaves of <= 4: at least T/4 - 1 inner nodes, fewer than T
        assert st["triangles"] // 4 - st["meshes"] <= st["bvh_nodes"] < st["triangles"], st
        assert st["depth"] <= 64, st


def test_degenerate_mesh_is_deeper_than_the_search_stack(built):
    """The degenerate fixture (tests/golden/make_fixture_degenerate.py) builds a BVH deeper than the per-lane
    search stack (frt_engine.hip kMeshStackMax = 32): the upload caps the stack instead of growing every
    traversal block's LDS, and the searches fall back to the group walk where it is full (the GPU image
    equals the plain walk's: test_gpu_parity.py test_mesh_search_equals_generic_walk)."""
    from fast_ray_tracer_amd.runtime import mesh_check
    bad, st = mesh_check(load_scene("degenerate_mesh_48"))
    assert bad == 0 and st["depth"] > 32, st


def test_mesh_switch_off(built, monkeypatch):
    """FRT_MESH=0 (the A/B switch read at upload) leaves every scene on the plain walk."""
    from fast_ray_tracer_amd.runtime import mesh_check
    monkeypatch.setenv("FRT_MESH", "0")
    bad, st = mesh_check(load_scene("bounding_boxes_100x125_4x4"))
    assert bad == 0 and st["meshes"] == 0, st
