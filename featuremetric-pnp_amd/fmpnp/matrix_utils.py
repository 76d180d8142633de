"""Rotation-matrix -> quaternion for the adapter's output (s2dhm/pose_prediction/matrix_utils.py:29-74).

Host-side numpy on a 4x4 matrix (one call per query, after the device loop).
Quaternion order (w, x, y, z), w >= 0, computed from the trace when it dominates
M[3,3] and otherwise from the largest diagonal element (Shoemake's method, the
`isprecise=True` form the adapter uses).
"""
import math

import numpy as np


def matrix_quaternion(matrix, isprecise=True):
    M = np.array(matrix, dtype=np.float64)[:4, :4]
    if not isprecise:
        # eigenvector form: quaternion = dominant eigenvector of the symmetric 4x4 K
        m = M
        Km = np.array([[m[0, 0] - m[1, 1] - m[2, 2], 0.0, 0.0, 0.0],
                       [m[0, 1] + m[1, 0], m[1, 1] - m[0, 0] - m[2, 2], 0.0, 0.0],
                       [m[0, 2] + m[2, 0], m[1, 2] + m[2, 1], m[2, 2] - m[0, 0] - m[1, 1], 0.0],
                       [m[2, 1] - m[1, 2], m[0, 2] - m[2, 0], m[1, 0] - m[0, 1], m[0, 0] + m[1, 1] + m[2, 2]]]) / 3.0
        w, V = np.linalg.eigh(Km)
        q = V[[3, 0, 1, 2], np.argmax(w)]
    else:
        tr = np.trace(M)
        q = np.empty(4)
        if tr > M[3, 3]:
            q[0] = tr
            q[1] = M[2, 1] - M[1, 2]
            q[2] = M[0, 2] - M[2, 0]
            q[3] = M[1, 0] - M[0, 1]
            norm_t = tr
        else:
            # largest diagonal element i, with (j, k) the cyclic successors
            i = 0
            if M[1, 1] > M[0, 0]:
                i = 1
            if M[2, 2] > M[i, i]:
                i = 2
            j, k = (i + 1) % 3, (i + 2) % 3
            norm_t = M[i, i] - (M[j, j] + M[k, k]) + M[3, 3]
            v = np.empty(3)
            v[i] = norm_t
            v[j] = M[i, j] + M[j, i]
            v[k] = M[k, i] + M[i, k]
            q[0] = M[k, j] - M[j, k]
            q[1:] = v
        q *= 0.5 / math.sqrt(norm_t * M[3, 3])
    if q[0] < 0.0:
        q = -q
    return q
