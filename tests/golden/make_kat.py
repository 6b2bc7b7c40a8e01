"""Generate tests/golden/kat_matlab.json from the reference's own known-answer quiz.

The reference's only known-answer data is the MATLAB self-evaluation quiz in a comment of
slam_ros/Robot.h:146-178 (duplicated at Robot.cpp:1189-1221): inputs and formulas for the
generic EKF uncertainty propagation and update step. This script evaluates exactly those
formulas (numpy float64) on exactly those inputs and stores inputs + outputs. It does not read
the reference at run time; the inputs below are transcribed from Robot.h:151-154, 167-172.
"""
import json
import os

import numpy as np

# UNCEARTAINITY PROPAGATION, Robot.h:146-156: P_prior = Fx*P*Fx' + Fu*Q*Fu'
Fx = np.array([[2.0, 1.0], [1.0, 2.0]])
Fu = np.array([[2.0, 1.0], [1.0, 2.0]])
P = np.eye(2)
Q = np.array([[0.5, 0.0], [0.0, 0.5]])
P_prior = Fx @ P @ Fx.T + Fu @ Q @ Fu.T

# UPDATE STEP, Robot.h:158-178
z = np.array([1.1, 1.9])
h = np.array([1.0, 2.0])
Hx = np.array([[2.0, 1.0], [1.0, 2.0]])
Pp = np.eye(2)
R = np.array([[0.5, 0.0], [0.0, 0.5]])
x_prior = np.array([1.0, 2.0])
y = z - h
S = Hx @ Pp @ Hx.T + R
K = Pp @ Hx @ np.linalg.inv(S)          # the quiz's K = P_prior*Hx*inv(S)
x_post = x_prior + K @ y
P_post = Pp - Pp @ Hx @ K.T              # the quiz's P_posterior

out = {
    "source": "slam_ros/Robot.h:146-178 (MATLAB quiz in a comment)",
    "propagation": {"Fx": Fx.tolist(), "Fu": Fu.tolist(), "P": P.tolist(), "Q": Q.tolist(),
                    "P_prior": P_prior.tolist()},
    "update": {"z": z.tolist(), "h": h.tolist(), "Hx": Hx.tolist(), "P_prior": Pp.tolist(),
               "R": R.tolist(), "x_prior": x_prior.tolist(), "y": y.tolist(), "S": S.tolist(),
               "K": K.tolist(), "x_posterior": x_post.tolist(), "P_posterior": P_post.tolist()},
}
path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat_matlab.json")
with open(path, "w") as f:
    json.dump(out, f, indent=1)
print(path)
