"""korali_amd — MI355X-native engine for Korali's population-based solver
generation loop (CMA-ES, TMCMC).  See DESIGN.md."""
__version__ = "0.1.0"
