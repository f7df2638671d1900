"""Alias of restnet_ddp.py with the typo fixed."""
from restnet_ddp import launch

if __name__ == "__main__":
    launch("ddp")
