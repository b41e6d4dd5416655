"""BoW-matcher test inputs (generators live in orb_slam_2_ros_amd.synth_match)."""
from orb_slam_2_ros_amd.synth_match import BOW_VARIANT_ARGS as VARIANT_ARGS  # noqa: F401
from orb_slam_2_ros_amd.synth_match import make_bow_case as make_case  # noqa: F401
