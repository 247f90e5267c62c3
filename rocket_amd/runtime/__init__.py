"""rocket_amd.runtime"""
