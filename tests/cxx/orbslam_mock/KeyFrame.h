// Test stand-in: the reference splits these classes over several headers.
#pragma once
#include "Frame.h"
