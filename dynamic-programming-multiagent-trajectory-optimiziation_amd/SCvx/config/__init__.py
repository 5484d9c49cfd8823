"""Scenario data of the reference's SCvx/config package (default_scenario, default_game,
SI_default_scenario, SI_default_game): start / goal states, obstacles and game weights used by the
example drivers and the reference-pin runs.  Data only."""
