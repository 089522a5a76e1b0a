"""In-memory synthetic meshes for benchmarks (icosphere OBJ text)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def icosphere_obj(r, subdiv):
    from make_synthetic_ycb import convex_obj, icosphere_verts
    return convex_obj(icosphere_verts(r, subdiv), "icosphere")
