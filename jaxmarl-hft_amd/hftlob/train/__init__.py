"""Learners that consume the HIP env step (the reference's gymnax_exchange/jaxrl)."""
