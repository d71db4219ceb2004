from .env import MarineNavEnv3  # noqa: F401  (rfarl/rfarl/envs/marinenav/__init__.py:1)
