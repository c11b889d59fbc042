"""proto"""
