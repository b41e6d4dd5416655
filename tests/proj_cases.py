"""Projection-matcher test inputs (generators live in orb_slam_2_ros_amd.synth_match)."""
from orb_slam_2_ros_amd.synth_match import PROJ_VARIANT_ARGS as VARIANT_ARGS  # noqa: F401
from orb_slam_2_ros_amd.synth_match import make_proj_case as make_case  # noqa: F401
from orb_slam_2_ros_amd.synth_match import make_sim3_case  # noqa: F401
