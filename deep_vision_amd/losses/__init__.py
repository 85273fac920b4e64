"""losses"""
