"""Kinematic models of the dexterous hands for the contact sampler
(reference: mgs/sampler/kin/base.py, mgs/sampler/kin/shadow.py)."""
from mgs.sampler.kin.model import KinematicsModel, ShadowKinematicsModel, get_kinematics  # noqa: F401
