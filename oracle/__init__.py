"""Test infrastructure: CPU oracle for the FQL update (never imported by the product)."""
