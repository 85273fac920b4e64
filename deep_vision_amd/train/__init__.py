"""train"""
