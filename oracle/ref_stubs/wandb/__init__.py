"""Stub of wandb (absent here): onpolicy/runner/shared/base_runner.py imports it at module level;
the functions the fixtures call (process_infos, log_env with use_wandb=False) never touch it."""
