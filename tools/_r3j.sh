bash tools/profile.sh r3j "calib sq2 sq3 ta"
