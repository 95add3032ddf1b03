"""Drop-in for the reference's `fql` submodule surface (reference .gitmodules:1-4):
only what the in-tree callers import -- `fql.agents.fql.FQLAgent` and the
dataset helpers -- backed by the HIP population engine (fqlpop)."""
