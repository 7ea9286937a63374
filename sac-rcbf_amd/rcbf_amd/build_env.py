"""build_env (build_env.py:8-16) returning the device-backed envs."""
from .envs import SimulatedCarsEnv, UnicycleEnv


def build_env(args):
    """Build our custom gym environment."""
    if args.env_name == "Unicycle":
        return UnicycleEnv()
    elif args.env_name == "SimulatedCars":
        return SimulatedCarsEnv()
    else:
        raise Exception("Env {} not supported!".format(args.env_name))
