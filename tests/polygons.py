"""Non-rectangular test geometries (axis-parallel polygons, clockwise like the reference's
rectangle, Grid.cpp:28-72) shared by the CPU and GPU mask tests: vertices, x / y segment
specs (Grid.cpp:78-120 format: start, end, cells, ratio) and one (type, info) BC per edge."""
INLET, WALL, NEUMANN = 0, 2, 4

# backward-facing step: inlet on the upper half of x = 0, outflow at x = 2
STEP = dict(vertices=[(0, 0.5), (0, 1), (2, 1), (2, 0), (0.5, 0), (0.5, 0.5)],
            xspec=[[0, 2, 48, -1]], yspec=[[0, 1, 24, -1]],
            bc=[(INLET, 1.0), (WALL, 0.0), (NEUMANN, 0.0), (WALL, 0.0), (WALL, 0.0), (WALL, 0.0)])
# L-shaped lid-driven cavity (the lid is the top edge)
LSHAPE = dict(vertices=[(0, 0), (0, 1), (1, 1), (1, 0.5), (0.5, 0.5), (0.5, 0)],
              xspec=[[0, 1, 32, -1]], yspec=[[0, 1, 32, -1]],
              bc=[(WALL, 0.0), (WALL, 1.0), (WALL, 0.0), (WALL, 0.0), (WALL, 0.0), (WALL, 0.0)])
# a rectangle whose west side is two edges (inlet below, wall above): every cell inside, but
# not the four-edge rectangle of the fast path
SPLIT = dict(vertices=[(0, 0), (0, 0.5), (0, 1), (1, 1), (1, 0)],
             xspec=[[0, 1, 24, -1]], yspec=[[0, 1, 20, -1]],
             bc=[(INLET, 0.5), (WALL, 0.0), (WALL, 1.0), (NEUMANN, 0.0), (WALL, 0.0)])
# a stretched U-channel: inlet bottom-left, outflow bottom-right, around a central block
UCHAN = dict(vertices=[(0, 0), (0, 1), (1.5, 1), (1.5, 0), (1, 0), (1, 0.5), (0.5, 0.5), (0.5, 0)],
             xspec=[[0, 0.5, 10, 1.05], [0.5, 1.0, 12, -1], [1.0, 1.5, 10, 0.95]], yspec=[[0, 1, 24, -1]],
             bc=[(WALL, 0.0), (WALL, 0.0), (WALL, 0.0), (WALL, 0.0), (NEUMANN, 0.0), (WALL, 0.0), (WALL, 0.0),
                 (INLET, 1.0)])
# the L-shaped cavity on a stretched grid (walls only: the area-consistent Poisson rhs)
LSHAPE_S = dict(LSHAPE, xspec=[[0, 0.5, 12, 1.04], [0.5, 1, 12, 0.96]], yspec=[[0, 0.5, 10, 0.95], [0.5, 1, 14, -1]])
# (r5) the backward-facing step on a power-of-two box (64 x 32): its bounding box has the direct solve with the
# outflow elimination, so the GPU's Poisson solve is the bordered capacitance solve
STEP_P2 = dict(STEP, xspec=[[0, 2, 64, -1]], yspec=[[0, 1, 32, -1]])
ALL = {"step": STEP, "lshape": LSHAPE, "split": SPLIT, "uchannel": UCHAN, "lshape_s": LSHAPE_S, "step_p2": STEP_P2}
# (r6) larger boxes for the masked LDS-tiled kernels (64-column tiles, 2-cell ring in j): ny >= 128, so checked
# comparisons cross the column-tile boundaries; not in ALL (the per-kernel sets stay small)
LSHAPE_BIG = dict(LSHAPE, xspec=[[0, 1, 160, -1]], yspec=[[0, 1, 200, -1]])
STEP_BIG = dict(STEP, xspec=[[0, 2, 256, -1]], yspec=[[0, 1, 136, -1]])
BIG = {"lshape_big": LSHAPE_BIG, "step_big": STEP_BIG}
