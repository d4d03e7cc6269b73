"""ORACLE — test infrastructure only (see mpn_ref.py). Not part of the product."""
