"""Writes reference_known_answers.json: the known-answer vectors that the
reference's own unit tests hold for this path, transcribed as data (inputs
and expected outputs) with the file:line each one comes from.

    python tests/golden/make_reference_vectors.py

Sources (AlainSchoebi/semantic-bundle-adjustment-colmap, read as text):
  src/base/cost_functions_test.cc:41-99
  src/base/projection_test.cc:95-124
  src/base/camera_models_test.cc:39-218
  src/optim/bundle_adjustment_test.cc:186-642
"""
import json
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_known_answers.json")

cost_function = {
    "source": "src/base/cost_functions_test.cc:41-99",
    "model": "SIMPLE_PINHOLE",
    "observed": [0.0, 0.0],
    "qvec": [1, 0, 0, 0],
    "tvec": [0, 0, 0],
    # (point3D, camera_params) -> residuals; same for the constant-pose functor
    "cases": [
        {"point3D": [0, 0, 1], "camera": [1, 0, 0], "residual": [0, 0]},
        {"point3D": [0, 1, 1], "camera": [1, 0, 0], "residual": [0, 1]},
        {"point3D": [0, 1, 1], "camera": [2, 0, 0], "residual": [0, 2]},
        {"point3D": [-1, 1, 1], "camera": [2, 0, 0], "residual": [-2, 2]},
    ],
}

projection = {
    "source": "src/base/projection_test.cc:95-124",
    "model": "SIMPLE_PINHOLE",
    "camera": [1, 0, 0],
    "qvec": [1, 0, 0, 0],
    "tvec": [0, 0, 0],
    # error of the exact projection is 0; shifting the observation by (+1,+1) gives 2
    "shift_error": 2.0,
    "close_tol_percent": 1e-6,
}

camera_models = {
    "source": "src/base/camera_models_test.cc:39-218",
    "world_grid": {"start": -0.5, "stop": 0.5, "step": 0.1, "tol": 1e-6},
    "image_grid": {"start": 0, "stop": 800, "step": 50, "tol": 1e-6},
    "models": {
        "SIMPLE_PINHOLE": [[655.123, 386.123, 511.123]],
        "PINHOLE": [[651.123, 655.123, 386.123, 511.123]],
        "SIMPLE_RADIAL": [[651.123, 386.123, 511.123, 0.0], [651.123, 386.123, 511.123, 0.1]],
        "RADIAL": [[651.123, 386.123, 511.123, 0.0, 0.0], [651.123, 386.123, 511.123, 0.1, 0.0],
                   [651.123, 386.123, 511.123, 0.05, 0.0], [651.123, 386.123, 511.123, 0.05, 0.03]],
        "OPENCV": [[651.123, 655.123, 386.123, 511.123, -0.471, 0.223, -0.001, 0.001]],
    },
}

# GenerateReconstruction(num_images, num_points) -> config -> pinned summary counts
bundle_adjustment = {
    "source": "src/optim/bundle_adjustment_test.cc:186-642",
    "model": "SIMPLE_RADIAL",
    "cases": [
        {"name": "TestConfigNumObservations", "line": "186-208", "images": 4, "points": 100,
         "steps": [{"add_images": [0, 1], "num_residuals": 400},
                   {"add_variable_points": [1], "num_residuals": 404},
                   {"add_constant_points": [2], "num_residuals": 408},
                   {"add_images": [2], "num_residuals": 604},
                   {"add_images": [3], "num_residuals": 800}]},
        {"name": "TestTwoView", "line": "210-245", "images": 2, "points": 100, "config_images": [0, 1],
         "constant_pose": [0], "constant_tvec": {"1": [0]}, "num_residuals_reduced": 400,
         "num_effective_parameters_reduced": 309,
         "variable_cameras": [0, 1], "constant_images": [0], "constant_x_images": [1], "variable_points": "all"},
        {"name": "TestTwoViewConstantCamera", "line": "247-279", "images": 2, "points": 100,
         "config_images": [0, 1], "constant_pose": [0, 1], "constant_cameras": [0],
         "num_residuals_reduced": 400, "num_effective_parameters_reduced": 302,
         "variable_cameras": [1], "constant_image_cameras": [0], "constant_images": [0, 1], "variable_points": "all"},
        {"name": "TestPartiallyContainedTracks", "line": "281-326", "images": 3, "points": 100,
         "delete_observation": [2, 0], "config_images": [0, 1], "constant_pose": [0, 1],
         "num_residuals_reduced": 400, "num_effective_parameters_reduced": 7,
         "variable_cameras": [0, 1], "constant_image_cameras": [2], "variable_points": "deleted_only"},
        {"name": "TestPartiallyContainedTracksForceToOptimizePoint", "line": "328-387", "images": 3,
         "points": 100, "delete_observation": [2, 0], "config_images": [0, 1], "constant_pose": [0, 1],
         "add_variable_point_of": [2, 1], "add_constant_point_of": [2, 2],
         "num_residuals_reduced": 402, "num_effective_parameters_reduced": 10},
        {"name": "TestConstantPoints", "line": "389-432", "images": 2, "points": 100, "config_images": [0, 1],
         "constant_pose": [0, 1], "constant_points": [1, 2], "num_residuals_reduced": 400,
         "num_effective_parameters_reduced": 298},
        {"name": "TestVariableImage", "line": "434-477", "images": 3, "points": 100, "config_images": [0, 1, 2],
         "constant_pose": [0], "constant_tvec": {"1": [0]}, "num_residuals_reduced": 600,
         "num_effective_parameters_reduced": 317},
        {"name": "TestConstantFocalLength", "line": "479-525", "images": 2, "points": 100,
         "config_images": [0, 1], "constant_pose": [0], "constant_tvec": {"1": [0]},
         "options": {"refine_focal_length": 0}, "num_residuals_reduced": 400,
         "num_effective_parameters_reduced": 307},
        {"name": "TestVariablePrincipalPoint", "line": "527-585", "images": 2, "points": 100,
         "config_images": [0, 1], "constant_pose": [0], "constant_tvec": {"1": [0]},
         "options": {"refine_principal_point": 1}, "num_residuals_reduced": 400,
         "num_effective_parameters_reduced": 313},
        {"name": "TestConstantExtraParam", "line": "587-633", "images": 2, "points": 100,
         "config_images": [0, 1], "constant_pose": [0], "constant_tvec": {"1": [0]},
         "options": {"refine_extra_params": 0}, "num_residuals_reduced": 400,
         "num_effective_parameters_reduced": 307},
    ],
}

if __name__ == "__main__":
    with open(OUT, "w") as f:
        json.dump({"cost_function": cost_function, "projection": projection, "camera_models": camera_models,
                   "bundle_adjustment": bundle_adjustment}, f, indent=1)
    print("wrote", OUT)
